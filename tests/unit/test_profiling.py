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
