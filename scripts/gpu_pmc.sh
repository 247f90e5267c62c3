#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/pmc1 -- python $R/bench.py --no-graph --steps 5 --warmup 2 > $R/gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS -d $R/gpurun_out/pmc2 -- python $R/bench.py --no-graph --steps 5 --warmup 2 > $R/gpurun_out/pmc2.log 2>&1
echo done
