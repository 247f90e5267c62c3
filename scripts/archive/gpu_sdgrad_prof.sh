#!/bin/bash
# per-call conv kernel times of one ResNet-50 step, native vs library strided dgrad
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for mode in native lib; do
  ROCKET_CONV_SDGRAD=$mode bash scripts/gpu_rn50_prof.sh || exit 1
  mv gpurun_out/rn50_kernels.md gpurun_out/rn50_kernels_$mode.md
  mv gpurun_out/rn50_conv_calls.txt gpurun_out/rn50_conv_calls_$mode.txt
done
