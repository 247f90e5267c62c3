#!/bin/bash
# dense fp16 weight shadows maintained by the fused optimizers: tests, fp16/bf16 benches, LeNet headline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_ce_optim.py tests/gpu/test_launcher_gpu.py tests/kernels/test_amp.py tests/kernels/test_iconv.py -m gpu > gpurun_out/f16sh_tests.log 2>&1 || { tail -40 gpurun_out/f16sh_tests.log; exit 1; }
tail -1 gpurun_out/f16sh_tests.log
for a in "resnet18 fp16" "resnet50 fp16" "resnet18 bf16" "lenet bf16"; do set -- $a
  timeout -k 10 300 python bench.py --model $1 --mp $2 --steps 20 --warmup 5 > gpurun_out/f16sh_$1_$2.json 2> gpurun_out/f16sh_$1_$2.err || { tail -20 gpurun_out/f16sh_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/f16sh_$1_$2.json'));print('$1 $2',d['value'],d['ms_per_step'])"
done
