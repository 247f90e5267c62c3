"""Phase timeline of the fused LeNet forward / backward launches (diagnostics).

    python bench/lenet_timeline.py [--batch 1024] [--steps 20]

Runs fused LeNet training steps (forward, fused cross-entropy + backward) with the kernels'
phase stamps enabled (``rk_lenet_set_trace``): thread 0 of every block records
``s_memrealtime`` (100 MHz) at each phase boundary.  Prints, per phase, the median over blocks
of the time since the previous stamp and of the time since the launch's earliest block start,
averaged over the last steps — where a latency-chain kernel spends its time.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

FWD = ["start", "stage img + w1", "conv1 tiles (wave 0)", "w2 frags + sync", "a1/code1 stores", "conv2 + sync",
       "fc1 + sync", "fc2 + sync", "fc3 (end)"]
BWD = ["start", "wfr + CE loads + sync", "stage issue (dc2/dcT zero)", "CE softmax + sync", "fc3 dgrad + sync",
       "fc2 dgrad + sync", "fc1 dgrad + sync", "scatter + sync", "conv2 dgrad + sync", "dW1/dW2 MFMA (wave 0)",
       "dW2 partials out + sync", "dW1 partials out", "CE loss partials (end)"]
BWD_MARKS = [0, 1, 2, 3, 5, 6, 7, 8, 9, 13, 10, 11, 12]


def summarize(tr: torch.Tensor, names, marks):
    t = tr[:, marks].double()
    t0 = t[:, 0].min()
    rows = []
    for j, k in enumerate(marks):
        col = t[:, j]
        since0 = float((col - t0).median()) * 10.0 / 1e3  # 100 MHz ticks -> us
        d = float((col - t[:, j - 1]).median()) * 10.0 / 1e3 if j else float((col - t0).median()) * 10.0 / 1e3
        rows.append({"phase": names[j], "median_us_since_prev": round(d, 2), "median_us_since_launch": round(since0, 2),
                     "max_us_since_launch": round(float((col - t0).max()) * 10.0 / 1e3, 2)})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    from rocket_amd import ops
    from rocket_amd.models import LeNet
    from rocket_amd.ops import _lib
    from rocket_amd.ops.lenet import fuse_cross_entropy

    ops.set_fused(True)
    lib = _lib.kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = LeNet(fused=True).to(dev)
    x = torch.rand(a.batch, 1, 28, 28, device=dev)
    y = torch.randint(0, 10, (a.batch,), device=dev)
    blocks = a.batch // 4
    ftr = torch.zeros(blocks, 48, dtype=torch.int64, device=dev)
    btr = torch.zeros(blocks, 48, dtype=torch.int64, device=dev)
    lib.rk_lenet_set_trace(ftr.data_ptr(), btr.data_ptr())
    fw, bw, waves = [], [], []
    try:
        for step in range(a.steps):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits = net.logits(x)
            loss, g = fuse_cross_entropy(logits, y, 1.0)
            torch.autograd.backward([logits], [g])
            net.zero_grad(set_to_none=False)
            torch.cuda.synchronize()
            if step >= a.steps // 2:
                fw.append(summarize(ftr.cpu(), FWD, list(range(9))))
                bw.append(summarize(btr.cpu(), BWD, BWD_MARKS))
                b = btr.cpu().double()
                start = b[:, 8:9]  # after scatter + sync: phase B begins
                waves.append({"dW2_done_us": ((b[:, 16:26] - start).median(0).values * 0.01).tolist(),
                              "dgrad_done_us": ((b[:, 32:48] - start).median(0).values * 0.01).tolist()})
    finally:
        lib.rk_lenet_set_trace(None, None)

    def avg(runs):
        out = []
        for j in range(len(runs[0])):
            r = dict(runs[0][j])
            for k in ("median_us_since_prev", "median_us_since_launch", "max_us_since_launch"):
                r[k] = round(statistics.mean(run[j][k] for run in runs), 2)
            out.append(r)
        return out

    print(json.dumps({"kernel": "lenet_fwd", "batch": a.batch, "phases": avg(fw)}))
    print(json.dumps({"kernel": "lenet_bwd", "batch": a.batch, "phases": avg(bw)}))
    n = len(waves)
    print(json.dumps({"kernel": "lenet_bwd phase B per wave (us after phase start, median over blocks)",
                      "dW2_done": [round(sum(w["dW2_done_us"][i] for w in waves) / n, 2) for i in range(10)],
                      "dgrad_done": [round(sum(w["dgrad_done_us"][i] for w in waves) / n, 2) for i in range(16)]}))


class StepTrace:
    """Phase stamps of the CAPTURED bench step (``ROCKET_LENET_TRACE=<file>`` in bench.py): the
    stamp buffers are installed before the step is captured, so every replay of the graph writes
    them and the last step's stamps remain.  All stamps share one clock (s_memrealtime, 100 MHz),
    so the launches' spans and the gaps between them come out on one time axis."""

    def __init__(self, batch: int):
        from rocket_amd.ops import _lib

        self.lib = _lib.kernels()
        dev = torch.device("cuda", 0)
        blocks = batch // 4
        self.ftr = torch.zeros(blocks, 48, dtype=torch.int64, device=dev)
        self.btr = torch.zeros(blocks, 48, dtype=torch.int64, device=dev)
        self.wtr = torch.zeros(512, 8, dtype=torch.int64, device=dev)
        self.lib.rk_lenet_set_trace(self.ftr.data_ptr(), self.btr.data_ptr())
        self.lib.rk_mlp3_set_trace(self.wtr.data_ptr())
        self.gtr = torch.zeros(4096, 2, dtype=torch.int64, device=dev)
        self.lib.rk_gather_set_trace(self.gtr.data_ptr())

    def report(self) -> dict:
        torch.cuda.synchronize()
        self.lib.rk_lenet_set_trace(None, None)
        self.lib.rk_mlp3_set_trace(None)
        self.lib.rk_gather_set_trace(None)
        f, b = self.ftr.cpu().double(), self.btr.cpu().double()
        w = self.wtr.cpu().double()
        w = w[w[:, 0] > 0]
        t0 = f[:, 0].min()
        us = lambda v: round(float(v - t0) * 0.01, 2)  # noqa: E731
        spans = {
            "fwd": {"first_start": us(f[:, 0].min()), "median_end": us(f[:, 8].median()), "last_end": us(f[:, 8].max())},
            "bwd": {"first_start": us(b[:, 0].min()), "median_end": us(b[:, 12].median()), "last_end": us(b[:, 12].max())},
            "wgrad": {"first_start": us(w[:, 0].min()), "median_loads_done": us(w[:, 1][w[:, 1] > 0].median()),
                      "median_end": us(w[:, 2].median()), "last_end": us(w[:, 2].max()), "blocks": int(w.shape[0])},
        }
        wall = self.wtr.cpu().double()
        # block ranges of the grouped launch (mlp.hip: 16 x 32 dW tiles, 32-column slab blocks)
        groups = {"fc3 tiles": (0, 3), "fc2 tiles": (3, 27), "fc1 tiles": (27, 131), "slab cols": (131, 212),
                  "loss": (212, 213)}
        wg = {}
        for name, (lo, hi) in groups.items():
            g = wall[lo:hi]
            if g.shape[0] and float(g[:, 0].min()) > 0:
                wg[name] = {"median_start": us(g[:, 0].median()), "median_reduced": us(g[:, 1].median()),
                            "median_end": us(g[:, 2].median()), "last_end": us(g[:, 2].max())}
                if float(g[:, 3].min()) > 0:
                    wg[name]["median_old_loaded"] = us(g[:, 3].median())
                    wg[name]["median_loop_done"] = us(g[:, 4].median())
        spans["wgrad_groups"] = wg
        g = self.gtr.cpu().double()
        g = g[g[:, 0] > 0]
        if g.shape[0]:  # the NEXT batch's gather (issued one ahead, before this step's launches)
            spans["next_batch_gather"] = {"first_start": us(g[:, 0].min()), "last_end": us(g[:, 1].max()),
                                          "blocks": int(g.shape[0])}
        # per-wave stamps (us after the block's own phase start, median over blocks, per wave)
        per_wave = lambda tr, cols, ref: [round(float(v) * 0.01, 2) for v in (tr[:, cols] - tr[:, ref:ref + 1]).median(0).values]  # noqa: E731
        waves = {"fwd conv1 done (after staging)": per_wave(f, slice(16, 32), 1),
                 "fwd conv2 done (after the conv1 barrier)": per_wave(f, slice(32, 48), 3),
                 "bwd dW2 tile done (after scatter)": per_wave(b, slice(16, 26), 8),
                 "bwd dgrad tiles done (after scatter)": per_wave(b, slice(32, 48), 8)}
        return {"kernel": "captured LeNet step (us from the forward's first block start)", "spans": spans,
                "fwd_phases": summarize(self.ftr.cpu(), FWD, list(range(9))),
                "bwd_phases": summarize(self.btr.cpu(), BWD, BWD_MARKS), "waves": waves}


if __name__ == "__main__":
    main()
