#!/bin/bash
# BN elementwise passes with SGPR-based 32-bit offsets: BN numerics, ResNet benches + BN kernel times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_norm.py \
  tests/kernels/test_fp16.py tests/kernels/test_iconv.py tests/gpu/test_model_parity.py > gpurun_out/r4m_tests.log 2>&1 || { tail -30 gpurun_out/r4m_tests.log; exit 1; }
tail -2 gpurun_out/r4m_tests.log
for i in 1 2; do
for m in resnet50 resnet18; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r4m_$m.json 2>/dev/null || exit 1
  echo "$m $(python3 -c "import json;r=json.loads(open('gpurun_out/r4m_$m.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")"
done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4m_rn50 -o run -- python3 $R/bench.py --model resnet50 --steps 6 --warmup 3 > $R/gpurun_out/r4m_rn50_trace.log 2>&1 || { tail -20 $R/gpurun_out/r4m_rn50_trace.log; exit 1; }
cd $R
f=$(find gpurun_out/r4m_rn50 -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 3 --title "ResNet-50 bs256 bf16 step (round 4), rocprofv3 kernel trace" > gpurun_out/r4_resnet50_kernels.md
rm -rf gpurun_out/r4m_rn50
head -24 gpurun_out/r4_resnet50_kernels.md
