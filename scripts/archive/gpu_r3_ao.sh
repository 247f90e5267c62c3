#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r3g; export TMPDIR=/tmp
timeout -k 10 120 python bench/gap_probe.py > gpurun_out/r3g/anyorder.jsonl 2>gpurun_out/r3g/anyorder.err || { tail -20 gpurun_out/r3g/anyorder.err; exit 1; }
head -3 gpurun_out/r3g/anyorder.jsonl
