#!/bin/bash
# LDS-staged conv epilogue: numerics, ResNet benches (on vs ROCKET_CONV_LDS_EPI=0), ResNet-50 trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_iconv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/epi_tests.log 2>&1 || exit 1
for m in resnet50 resnet18; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/epi_$m.json 2> gpurun_out/epi_$m.err || exit 1
  ROCKET_CONV_LDS_EPI=0 timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/epi_${m}_off.json 2> gpurun_out/epi_${m}_off.err || exit 1
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/epi_${m}_2.json 2> gpurun_out/epi_${m}_2.err || exit 1
done
MODEL=resnet50 bash scripts/gpu_rn50_prof.sh
