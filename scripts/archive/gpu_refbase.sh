#!/bin/bash
# Reference pipeline on 1x MI355X with GPU-resident synthetic data and with
# the host TensorDataset, bf16 and fp32 -> gpurun_out/refbase.jsonl
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out; : > gpurun_out/refbase.jsonl
[ -d _refbase/rocket ] || bash scripts/make_refbase.sh
for args in "--mp bf16 --device-data" "--mp no --device-data" "--mp bf16" ; do
  timeout -k 10 240 python bench/reference_baseline.py --steps 100 --warmup 20 $args 2> gpurun_out/refbase.err | tail -1 >> gpurun_out/refbase.jsonl || exit 1
done
cat gpurun_out/refbase.jsonl
