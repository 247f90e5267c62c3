#!/bin/bash
# First GPU pass: kernel tests, reference baseline, torch-path bench, rocprof of torch path.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.get_device_name(0), torch.version.hip)" > gpurun_out/dev.txt 2>&1
timeout -k 10 400 python -m pytest tests/kernels -m gpu -x -q > gpurun_out/pytest_kernels.log 2>&1; echo "pytest rc=$?" >> gpurun_out/summary.txt
timeout -k 10 300 python bench/reference_baseline.py --steps 60 --warmup 10 --mp bf16 > gpurun_out/ref_bf16.json 2> gpurun_out/ref_bf16.err || exit 1
timeout -k 10 300 python bench/reference_baseline.py --steps 60 --warmup 10 --mp no > gpurun_out/ref_fp32.json 2> gpurun_out/ref_fp32.err || exit 1
timeout -k 10 300 python bench.py --impl torch --steps 100 --warmup 10 > gpurun_out/bench_torch.json 2> gpurun_out/bench_torch.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_torch -- python $R/bench.py --impl torch --steps 30 --warmup 5 > $R/gpurun_out/prof_torch.log 2>&1
echo "prof rc=$?" >> $R/gpurun_out/summary.txt
