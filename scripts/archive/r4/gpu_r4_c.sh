#!/bin/bash
# one-wave-per-SIMD GEMM probe (numerics + speed vs hipBLASLt / mgemm t0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python -u bench/xgemm4_probe.py > gpurun_out/xgemm4_probe.log 2>&1; rc=$?
cat gpurun_out/xgemm4_probe.log | grep -v amdgpu.ids
exit $rc
