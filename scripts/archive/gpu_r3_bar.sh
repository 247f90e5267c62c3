#!/bin/bash
# LDS-only barriers in the conv epilogue and the LeNet backward phases: tests + benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/kernels/test_linear_conv.py tests/kernels/test_ce_optim.py tests/kernels/test_iconv.py tests/gpu/test_graph_capture.py tests/gpu/test_device_loader_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/bar_tests.log 2>&1 || { tail -30 gpurun_out/bar_tests.log; exit 1; }
tail -1 gpurun_out/bar_tests.log
for i in 1 2; do
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bar_lenet20_$i.json 2> gpurun_out/bar_lenet20.err || exit 1
python -c "import json;r=json.load(open('gpurun_out/bar_lenet20_$i.json'));print('lenet20',r['value'],r['ms_per_step'],r['step_ms_p50'])"
done
timeout -k 10 120 python bench.py > gpurun_out/bar_lenet.json 2> gpurun_out/bar_lenet.err || exit 1
python -c "import json;r=json.load(open('gpurun_out/bar_lenet.json'));print('lenet1000',r['value'],r['ms_per_step'],r['step_ms_p50'])"
for m in resnet18 resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/bar_$m.json 2> gpurun_out/bar_$m.err || exit 1
  python -c "import json;r=json.load(open('gpurun_out/bar_$m.json'));print('$m',r['value'],r['ms_per_step'])"
done
