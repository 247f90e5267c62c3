"""FusedGradScaler's skip-flag ring (runtime/amp.py): the host-side publication used when an update
runs outside the fused kernel, handle resolution by update number, and the 31-bit sequence
encoding across the int32 wrap (the kernel stores (n << 1) | skipped as one 32-bit word)."""

import torch

from rocket_amd.runtime.amp import RING, SEQ, FusedGradScaler


def test_host_published_flags_resolve_per_update():
    sc = FusedGradScaler("cpu")
    handles = []
    for skipped in (False, True, False):
        sc._record_last(host_flag=skipped)
        handles.append(sc.last_handle())
    assert [FusedGradScaler.handle_ready(h) for h in handles] == [True, True, True]
    assert [FusedGradScaler.handle_skipped(h) for h in handles] == [False, True, False]
    assert int(sc.state.view(torch.int32)[SEQ]) == 3  # the device count follows host-run updates
    assert sc.last_step_skipped() is False


def test_no_update_yet_reads_not_skipped():
    sc = FusedGradScaler("cpu")
    h = sc.last_handle()
    assert FusedGradScaler.handle_ready(h) and FusedGradScaler.handle_skipped(h) is False


def test_sequence_encoding_across_int32_wrap():
    sc = FusedGradScaler("cpu")
    sc._seq = (1 << 31) - 2
    flags = [True, False, True, True]
    handles = []
    for f in flags:
        sc._record_last(host_flag=f)
        handles.append(sc.last_handle())
    assert [sc._entry(h[1]) for h in handles] == flags
    # an entry overwritten RING updates later no longer answers for the old update number
    old = handles[0][1]
    for _ in range(RING):
        sc._record_last(host_flag=False)
    assert sc._entry(old) is None
