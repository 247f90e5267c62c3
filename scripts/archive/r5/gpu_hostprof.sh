#!/bin/bash
# round 5: host-side profile (cProfile) of the LeNet step loop: 1000- and 5000-step runs per
# precision, so the difference (steady-state per-step cost) cancels the one-time setup / capture
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5hp; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
for mp in fp16 bf16; do
  for n in 1000 5000; do
    timeout -k 10 300 python -m cProfile -o $O/${mp}_$n.prof bench.py --mp $mp --steps $n --warmup 50 > $O/${mp}_$n.json 2>> $O/err.log || exit 1
  done
done
echo done
