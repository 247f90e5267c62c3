#!/bin/bash
# round 5 box t: LeNet tests/benches/timeline (gpu_h.sh), then LDS-conflict counters of the whole-step
# and the split (ROCKET_LENET_SPEC=0) launches at HEAD
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
RUN=${RUN:-r5t} bash $R/scripts/archive/r5/gpu_h.sh || exit 1
O=$R/gpurun_out/${RUN:-r5t}
cd /tmp && export TMPDIR=/tmp
B="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for p in A B; do
  ROCKET_LENET_SPEC=0 timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc ${!p} -d $O/s$p -o run -- python3 $R/bench.py --steps 30 --warmup 10 > $O/s$p.log 2>&1 || { echo "pmc $p failed"; tail -5 $O/s$p.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc ${!p} -d $O/w$p -o run -- python3 $R/bench.py --steps 30 --warmup 10 > $O/w$p.log 2>&1 || { echo "pmc $p failed"; tail -5 $O/w$p.log; exit 1; }
done
cd $R
python3 bench/summarize_pmc.py $O/sA $O/sB --steps 10 --marker mlp3_wgrad_kernel --title "LeNet, forward and backward as separate launches (ROCKET_LENET_SPEC=0), PMC" > $O/pmc_split.md || true
python3 bench/summarize_pmc.py $O/wA $O/wB --steps 10 --marker mlp3_wgrad_kernel --title "LeNet whole-step (default), PMC at HEAD" > $O/pmc_whole.md || true
rm -rf $O/sA $O/sB $O/wA $O/wB
cat $O/pmc_split.md $O/pmc_whole.md
