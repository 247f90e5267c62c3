#!/bin/bash
# round 5 first box: GPU suite + smoke + driver-shaped LeNet bench + host cProfile of the LeNet run
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r5a; export TMPDIR=/tmp
O=gpurun_out/r5a
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider -rf > $O/pytest.log 2>&1; rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/lenet_driver.json 2> $O/lenet_driver.err || exit 1
cat $O/lenet_driver.json
ROCKET_BENCH_PROFILE=$O/lenet.prof timeout -k 10 180 python bench.py --steps 2000 --warmup 50 > $O/lenet_prof.json 2> $O/lenet_prof.err || exit 1
python -c "
import pstats; p=pstats.Stats('$O/lenet.prof.0'); p.sort_stats('tottime').print_stats(45)" > $O/lenet_prof_tottime.txt
python -c "
import pstats; p=pstats.Stats('$O/lenet.prof.0'); p.sort_stats('cumulative').print_stats(60)" > $O/lenet_prof_cum.txt
cat $O/lenet_prof.json
timeout -k 10 300 python bench/gemm_r5_probe.py --out $O/gemm_probe.jsonl > $O/gemm_probe.log 2>&1 || exit 1
cat $O/gemm_probe.jsonl
