"""All-reduce bus bandwidth vs message size (and RCCL channel count) across the GPUs of one node.

The DDP gradient buckets (parallel/ddp.py) are sized from this curve: on MI355X every GPU has
7 xGMI links of ~153 GB/s (point-to-point, no switch), so a ring all-reduce is bound per link and
reaches its plateau only for messages of several MiB; below that the P2P one-shot kernel
(parallel/p2p.py) wins.  Run one process per GPU:

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29511 bench/allreduce_sweep.py [--channels 0,16,32] [--out gpurun_out/ar.jsonl]

``--channels c`` re-runs the sweep in a child process with ``NCCL_MIN_NCHANNELS=NCCL_MAX_NCHANNELS=c``
(0 = RCCL's default).  Bus bandwidth follows the nccl-tests convention: algbw * 2 (W-1) / W.
With ``--cpu`` it runs on gloo (correctness/plumbing rehearsal only; no bandwidth meaning).
Rank 0 prints one JSON line per (channels, size, transport).
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sweep(args) -> None:
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    cpu = args.cpu
    if not cpu:
        torch.cuda.set_device(local)
    dist.init_process_group("gloo" if cpu else "nccl", rank=rank, world_size=world)
    dev = torch.device("cpu") if cpu else torch.device("cuda", local)
    p2p = None
    if not cpu and args.p2p:
        try:
            from rocket_amd.parallel.p2p import MAX_ELEMS, P2PAllReduce

            host = dist.new_group(backend="gloo")
            p2p = P2PAllReduce.create(MAX_ELEMS, group=host, device=dev)
        except Exception as e:  # noqa: BLE001 - report and sweep RCCL only
            if rank == 0:
                print(json.dumps({"p2p": "unavailable", "why": str(e)[:200]}), flush=True)
    sizes = [1 << s for s in range(args.min_log2, args.max_log2 + 1)]
    out = open(args.out, "a") if (rank == 0 and args.out) else None
    for nbytes in sizes:
        n = nbytes // 4
        x = torch.ones(n, dtype=torch.float32, device=dev)
        transports = [("rccl" if not cpu else "gloo", lambda: dist.all_reduce(x))]
        if p2p is not None and n <= p2p.cap:
            transports.append(("p2p", lambda: p2p.all_reduce_(x)))
        for name, fn in transports:
            for _ in range(args.warmup):
                fn()
            if not cpu:
                torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                fn()
            if not cpu:
                torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.iters
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = t.item()
            algbw = nbytes / dt / 1e9
            rec = {"channels": args.channels_now, "bytes": nbytes, "transport": name, "world": world,
                   "us": round(dt * 1e6, 2), "algbw_GBps": round(algbw, 2),
                   "busbw_GBps": round(algbw * 2 * (world - 1) / world, 2)}
            if rank == 0:
                print(json.dumps(rec), flush=True)
                if out:
                    out.write(json.dumps(rec) + "\n")
                    out.flush()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-log2", type=int, default=12)
    ap.add_argument("--max-log2", type=int, default=28)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--channels", default="0", help="comma list of RCCL channel counts (0 = default)")
    ap.add_argument("--channels-now", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--p2p", action="store_true", help="also time the P2P one-shot all-reduce")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    chans = [int(c) for c in args.channels.split(",")]
    if len(chans) == 1:
        args.channels_now = chans[0]
        if chans[0]:
            os.environ["NCCL_MIN_NCHANNELS"] = os.environ["NCCL_MAX_NCHANNELS"] = str(chans[0])
        sweep(args)
        return
    # several channel counts: one child per count (RCCL reads the variables at init); every rank
    # runs the same sequence, so the children of all ranks rendezvous on the same port in turn
    for c in chans:
        cmd = [sys.executable, os.path.abspath(__file__), "--channels", str(c), "--min-log2", str(args.min_log2),
               "--max-log2", str(args.max_log2), "--iters", str(args.iters), "--warmup", str(args.warmup)]
        cmd += (["--p2p"] if args.p2p else []) + (["--cpu"] if args.cpu else []) + (["--out", args.out] if args.out else [])
        rc = subprocess.call(cmd)
        if rc:
            sys.exit(rc)


if __name__ == "__main__":
    main()
