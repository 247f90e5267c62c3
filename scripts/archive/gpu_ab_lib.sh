#!/bin/bash
# A/B of two native builds in one tree: ab_old/ (ROCKET_LIBDIR) vs rocket_amd/_lib.  LeNet tests on
# the new build, phase timeline of each, then the driver-shaped and long LeNet benches alternated.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/summary_ablib.txt
: > $S
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/kernels/test_lenet_conv.py tests/kernels/test_lenet_fused.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $S
[ $rc -ne 0 ] && { tail -30 gpurun_out/ab_tests.log; exit 1; }
for v in old new; do
  if [ $v = old ]; then export ROCKET_LIBDIR=$R/ab_old; else unset ROCKET_LIBDIR; fi
  timeout -k 10 120 python bench/lenet_timeline.py > gpurun_out/tl_$v.jsonl 2> gpurun_out/tl_$v.err; rc=$?; echo "timeline $v rc=$rc" >> $S
  [ $rc -ne 0 ] && exit 1
done
for rep in 1 2; do for v in old new; do
  if [ $v = old ]; then export ROCKET_LIBDIR=$R/ab_old; else unset ROCKET_LIBDIR; fi
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/abd_${v}_$rep.json 2>/dev/null; rc=$?
  timeout -k 10 300 python bench.py > gpurun_out/abl_${v}_$rep.json 2>/dev/null; rc2=$?
  echo "$v rep$rep rc=$rc/$rc2 driver=$(python -c "import json;print(json.loads(open('gpurun_out/abd_${v}_$rep.json').read().splitlines()[-1])['value'])") long=$(python -c "import json;print(json.loads(open('gpurun_out/abl_${v}_$rep.json').read().splitlines()[-1])['value'])")" >> $S
  [ $rc -ne 0 ] && exit 1
done; done
cat $S
