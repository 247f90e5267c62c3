#!/bin/bash
# LeNet whole-step PMC with the memory columns: 4 passes (SQ x2, FETCH_SIZE, WRITE_SIZE + TCC hit/miss)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6pl; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
C="FETCH_SIZE GRBM_GUI_ACTIVE"
D="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for p in A B C D; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc ${!p} -d $O/w$p -o run -- python3 $R/bench.py --steps 30 --warmup 10 > $O/w$p.log 2>&1 || { echo "pmc $p failed"; tail -5 $O/w$p.log; exit 1; }
done
cd $R && python3 bench/summarize_pmc.py $O/wA $O/wB $O/wC $O/wD --steps 10 --marker mlp3_wgrad_kernel --title "LeNet bs1024 whole step (round 6 HEAD), PMC with memory counters" > $O/pmc_lenet.md
rm -rf $O/wA $O/wB $O/wC $O/wD
cat $O/pmc_lenet.md
