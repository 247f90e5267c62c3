#!/bin/bash
# LDS epilogue with prefetched side inputs (BN input / mask / old output): conv tests + ResNet benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/kernels/test_iconv.py tests/kernels/test_fp16.py tests/kernels/test_norm.py tests/gpu/test_model_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/epi_tests.log 2>&1 || { tail -30 gpurun_out/epi_tests.log; exit 1; }
tail -1 gpurun_out/epi_tests.log
for m in resnet18 resnet50 resnet18 resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/epi_$m.json 2> gpurun_out/epi_$m.err || exit 1
  python -c "import json;r=json.load(open('gpurun_out/epi_$m.json'));print('$m',r['value'],r['ms_per_step'])"
done
