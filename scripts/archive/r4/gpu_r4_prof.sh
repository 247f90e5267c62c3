#!/bin/bash
# Profiling batch: xgemm vs mgemm PMC at 4096^3, LeNet step timeline, LeNet PMC.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/r4prof; rm -rf $O; mkdir -p $O
pmc() {  # name counters cmd...
  local n=$1 c=$2; shift 2
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $c -d $O/$n -o run -- "$@" > $O/$n.log 2>&1
}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
B="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
C="TCC_HIT_sum TCC_MISS_sum TCC_BUSY_sum GRBM_GUI_ACTIVE"
pmc gA "$A" python3 $R/bench/mgemm_one.py sq:fwd:20 sq:fwd:0 --M 4096 &&
pmc gB "$B" python3 $R/bench/mgemm_one.py sq:fwd:20 sq:fwd:0 --M 4096 &&
pmc gC "$C" python3 $R/bench/mgemm_one.py sq:fwd:20 sq:fwd:0 --M 4096 || { echo "gemm pmc failed"; exit 1; }
cd $R && python3 bench/summarize_pmc.py $O/gA $O/gB $O/gC --steps 1 --marker __none__ --top 10 --title "xgemm t20 vs mgemm t0 at 4096^3, PMC" > gpurun_out/r4_pmc_xgemm.md
cd $R && ROCKET_LENET_TRACE=gpurun_out/r4_lenet_timeline.json timeout -k 10 120 python bench.py --steps 200 --warmup 20 > gpurun_out/r4_lenet_trace_bench.json 2>gpurun_out/r4_lenet_trace.err || { echo "lenet trace failed"; exit 1; }
cd /tmp
pmc lA "$A" python3 $R/bench.py --no-graph --steps 10 --warmup 3 &&
pmc lB "$B" python3 $R/bench.py --no-graph --steps 10 --warmup 3 || { echo "lenet pmc failed"; exit 1; }
cd $R && python3 bench/summarize_pmc.py $O/lA $O/lB --steps 5 --marker mlp3_wgrad_kernel --title "LeNet bs1024 fused step (eager launches), PMC" > gpurun_out/r4_pmc_lenet.md
rm -rf $O/gA $O/gB $O/gC $O/lA $O/lB
cat gpurun_out/r4_pmc_xgemm.md gpurun_out/r4_pmc_lenet.md
