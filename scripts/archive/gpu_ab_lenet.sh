#!/bin/bash
# GPU tests + LeNet bench A/B over an env toggle: AB_VAR=name (values 0 and 1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/summary_ab.txt
: > $S
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
for rep in 1 2; do for v in 0 1; do
env $AB_VAR=$v timeout -k 10 300 python bench.py > gpurun_out/ab_${v}_$rep.json 2> gpurun_out/ab_${v}_$rep.err; rc=$?; echo "$AB_VAR=$v rep$rep rc=$rc" >> $S
[ $rc -ne 0 ] && exit 1
done; done
exit 0
