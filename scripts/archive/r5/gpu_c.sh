#!/bin/bash
# round 5 box c: LeNet KeepSmem (fwd state resident in LDS for the fused backward) - kernel tests,
# driver bench + long bench + step timeline; x4 GEMM with the LDS-staged epilogue (probe + stamps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5c; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_linear_conv.py \
  tests/kernels/test_fp16.py tests/kernels/test_amp.py tests/kernels/test_ce_optim.py tests/gpu/test_graph_capture.py \
  tests/gpu/test_launcher_gpu.py tests/examples > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/lenet_driver.json 2> $O/lenet_driver.err || exit 1
timeout -k 10 120 python bench.py --steps 1000 --warmup 50 > $O/lenet_long.json 2> $O/lenet_long.err || exit 1
ROCKET_LENET_TRACE=$O/lenet_timeline.json timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $O/lenet_trace_bench.json 2>$O/lenet_trace.err || exit 1
for f in lenet_driver lenet_long lenet_trace_bench; do python3 -c "import json;r=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', r['value'], r['ms_per_step'], r['step_ms_p50'], r['host_issue_ms'])"; done
timeout -k 10 200 python bench/x4_trace.py --out $O/x4_trace.json > $O/x4_trace.log 2>&1 || { tail -20 $O/x4_trace.log; exit 1; }
grep -v amdgpu.ids $O/x4_trace.log | cut -c1-400
timeout -k 10 300 python bench/gemm_r5_probe.py --out $O/gemm_probe.jsonl > $O/gemm_probe.log 2>&1 || { tail -20 $O/gemm_probe.log; exit 1; }
cat $O/gemm_probe.jsonl
