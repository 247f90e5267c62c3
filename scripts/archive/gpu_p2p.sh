#!/bin/bash
# P2P all-reduce kernel + DDP graph tests (2 ranks sharing the GPU)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/gpu/test_p2p.py tests/gpu/test_ddp_graph.py -q -m gpu -x > gpurun_out/p2p.log 2>&1; rc=$?
tail -30 gpurun_out/p2p.log
exit $rc
