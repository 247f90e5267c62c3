#!/bin/bash
# PMC passes over the LeNet step only (eager launches so every kernel is attributed), summarized on the box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmc_l; rm -rf $O; mkdir -p $O
run() { timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $2 -d $O/$1 -o run -- python3 $R/bench.py --no-graph --steps 10 --warmup 3 > $O/$1.log 2>&1; }
run A "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" &&
run B "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU" || exit 1
cd $R && python3 bench/summarize_pmc.py $O/A $O/B --steps 5 --marker mlp3_wgrad_kernel --title "LeNet bs1024 fused step (eager launches, AdamW fused into wgrad), PMC" > $R/gpurun_out/pmc_lenet_now.md
rc=$?; rm -rf $O/A $O/B; exit $rc
