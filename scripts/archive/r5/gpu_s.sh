#!/bin/bash
# round 5 box s: LDS bank conflicts / VALU / MFMA per LeNet kernel with the forward and backward as
# separate launches (ROCKET_LENET_SPEC=0), to locate the whole-step kernel's conflicts
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5s; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for p in A B; do
  ROCKET_LENET_SPEC=0 timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc ${!p} -d $O/s$p -o run -- python3 $R/bench.py --steps 30 --warmup 10 > $O/s$p.log 2>&1 || { echo "pmc $p failed"; tail -5 $O/s$p.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc ${!p} -d $O/w$p -o run -- python3 $R/bench.py --steps 30 --warmup 10 > $O/w$p.log 2>&1 || { echo "pmc $p failed"; tail -5 $O/w$p.log; exit 1; }
done
cd $R
python3 bench/summarize_pmc.py $O/sA $O/sB --steps 10 --marker mlp3_wgrad_kernel --title "LeNet, forward and backward as separate launches (ROCKET_LENET_SPEC=0), PMC" > gpurun_out/r5_pmc_lenet_progression.md || true
python3 bench/summarize_pmc.py $O/wA $O/wB --steps 10 --marker mlp3_wgrad_kernel --title "LeNet whole-step (default), PMC at HEAD" > gpurun_out/r5_pmc_lenet_progression.md || true
rm -rf $O/sA $O/sB $O/wA $O/wB
cat gpurun_out/r5_pmc_lenet_progression.md gpurun_out/r5_pmc_lenet_progression.md
