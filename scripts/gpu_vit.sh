#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/summary_vit.txt
timeout -k 10 300 python -m pytest tests/kernels/test_norm.py tests/gpu/test_models.py -q -m gpu -k "layernorm or vit" > gpurun_out/pytest_vit.log 2>&1; echo "pytest rc=$?" >> gpurun_out/summary_vit.txt
timeout -k 10 400 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/ab_vit_b16_fused.json 2> gpurun_out/ab_vit_b16_fused.err; echo "vit rc=$?" >> gpurun_out/summary_vit.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_vit -o run -- python3 bench.py --model vit_b16 --steps 10 --warmup 3 > gpurun_out/prof_vit.log 2>&1; echo "prof rc=$?" >> gpurun_out/summary_vit.txt
