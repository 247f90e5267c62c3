"""StepTimer grouping: with stride k the timer marks every k-th iteration and reports per-iteration
means of the groups (host-timestamp path, CPU)."""

import pytest

from rocket_amd.runtime.profiling import StepTimer


@pytest.mark.parametrize("steps,stride,expect", [(12, 4, [4, 4, 4]), (10, 4, [4, 4, 2]), (5, 1, [1] * 5)])
def test_group_sizes(steps, stride, expect):
    t = StepTimer(warmup=0, steps=steps, stride=stride)
    t._host = [0.0] * (len(expect) + 1)
    assert t._group_sizes() == expect


def test_step_times_are_per_iteration_means():
    t = StepTimer(warmup=0, steps=10, stride=4)
    # marks after iterations 0 (start), 4, 8, 10 -> groups of 4, 4, 2 iterations
    t._host = [0.0, 0.004, 0.008, 0.010]
    assert t.step_times_ms() == pytest.approx([1.0, 1.0, 1.0])
    assert t.host_ms_p50() == pytest.approx(1.0)


def test_tuned_gemm_table_is_valid_csv():
    """The shipped TunableOp table has the validator header and well-formed result rows."""
    import csv

    from rocket_amd.runtime.tuning import TABLE

    rows = list(csv.reader(open(TABLE)))
    assert rows[0][0] == "Validator" and any(r[1] == "GCN_ARCH_NAME" and r[2].startswith("gfx950") for r in rows
                                             if r[0] == "Validator")
    results = [r for r in rows if r[0] != "Validator"]
    assert results and all(len(r) == 4 and float(r[3]) > 0 for r in results)


def test_lenet_fragment_index_maps_cover_every_weight_once():
    """Every LeNet weight element has exactly one forward-layout slot in the fused kernels'
    fragment table (and fc / conv2 weights one input-gradient slot); no slot is shared."""
    import numpy as np

    from rocket_amd.ops.lenet import _NFRAG, _frag_index_maps

    maps = _frag_index_maps()
    slots = np.concatenate([m[m >= 0] for m in maps])
    assert len(np.unique(slots)) == len(slots) and slots.max() < _NFRAG * 64 * 8
    for name, m, has_bwd in zip(("fc1", "fc2", "fc3", "conv1", "conv2"), maps, (1, 1, 1, 0, 1)):
        assert (m[:, 0] >= 0).all(), name
        assert ((m[:, 1] >= 0).all() if has_bwd else (m[:, 1] < 0).all()), name


def test_lenet_conv2_dgrad_pixel_pair_decomposition():
    """Host model of the whole-step kernel's conv2 dgrad (lenet_conv.hip K2P / d2unit / phase B):
    A rows = pixel pairs, K = a 5 x 6 window of ring dConv2 pixels x 16 channels, columns (d, ci),
    B fragments gathered from the plain [kk][ci][co] table — equals the conv2 input gradient."""
    import numpy as np
    import torch

    from rocket_amd.ops.lenet import _OFF_D2, _frag_index_maps

    g = torch.Generator().manual_seed(0)
    w2 = torch.randn(16, 6, 5, 5, generator=g)
    dc = torch.randn(1, 16, 10, 10, generator=g)
    ref = torch.nn.grad.conv2d_input((1, 6, 14, 14), w2, dc)[0]  # [6][14][14]
    # the fragment table's dgrad section, written through the optimizer's index map
    table = np.zeros(282 * 64 * 8, dtype=np.float32)
    m = _frag_index_maps()[4][:, 1]
    table[m] = w2.numpy().reshape(-1)
    sect = table[_OFF_D2 * 512:].reshape(-1, 8)  # 16-byte units

    def d2unit(s, lane):
        h, c = lane >> 4, lane & 15
        pi = 2 * s + (h >> 1)
        dy, dx, d, ci = pi // 6, pi % 6, c >> 3, c & 7
        kh, kw = 4 - dy, 4 + d - dx
        return ((kh * 5 + kw) * 8 + ci) * 2 + (h & 1) if (0 <= kw < 5 and ci < 6) else -1

    B = np.zeros((15 * 32, 16), dtype=np.float32)  # B[k = 32s + 8hi + j][col lo]
    for s in range(15):
        for lane in range(64):
            u = d2unit(s, lane)
            if u >= 0:
                B[32 * s + 8 * (lane >> 4):32 * s + 8 * (lane >> 4) + 8, lane & 15] = sect[u]
    ring = np.zeros((18, 19, 16), dtype=np.float32)  # channel-last, zero ring of 4, 19-pixel row pitch
    ring[4:14, 4:14] = dc[0].permute(1, 2, 0).numpy()
    flat = ring.reshape(-1)
    out = np.full((6, 14, 14), np.nan, dtype=np.float32)

    def row_ih(r):  # tile row -> image row (14, 15: pad rows)
        return r + 4 if 4 <= r < 12 else (r if r < 4 else r - 8)

    for t in range(7):  # tile t = pixel pairs (ih, 2t .. 2t + 1)
        for r in range(16):
            ih = row_ih(r) if row_ih(r) < 14 else row_ih(r) - 8
            a = np.zeros(480, dtype=np.float32)
            for s in range(15):
                for hi in range(4):
                    base = ih * 304 + 2 * t * 16 + 8 * hi + (s // 3) * 304 + 2 * (s % 3) * 16
                    a[32 * s + 8 * hi:32 * s + 8 * hi + 8] = flat[base:base + 8]
            c = a @ B
            if row_ih(r) < 14:
                for lo in range(16):
                    if (lo & 7) < 6:
                        out[lo & 7, ih, 2 * t + (lo >> 3)] = c[lo]
    np.testing.assert_allclose(out, ref.numpy(), rtol=1e-4, atol=1e-4)
