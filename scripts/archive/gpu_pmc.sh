#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, --kernel-trace + --pmc only) over the LeNet
# step and the ResNet-50 / ViT-B/16 steps.  Counters absent from `rocprofv3 -L` are dropped.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmc; mkdir -p $O
timeout -s KILL 120 rocprofv3 -L > $O/counters.txt 2>&1 || exit 1
have() { local out=""; for c in "$@"; do grep -qw "$c" $O/counters.txt && out="$out $c"; done; echo $out; }
PA=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT)
PB=$(have SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL)
PC=$(have FETCH_SIZE TCC_HIT_sum)
PD=$(have WRITE_SIZE TCC_MISS_sum TCC_EA0_ATOMIC_sum)
echo "A: $PA" > $O/passes.txt; echo "B: $PB" >> $O/passes.txt; echo "C: $PC" >> $O/passes.txt; echo "D: $PD" >> $O/passes.txt
run() {  # name pass-counters timeout args...
  local name=$1 ctr=$2 to=$3; shift 3
  [ -z "$ctr" ] && return 0
  timeout -s KILL $to rocprofv3 --kernel-trace --output-format csv --pmc $ctr -d $O/$name -o run -- python3 $R/bench.py "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> $O/summary.txt; return $rc
}
: > $O/summary.txt
run lenet_A "$PA" 120 --no-graph --steps 10 --warmup 3 &&
run lenet_B "$PB" 120 --no-graph --steps 10 --warmup 3 &&
run lenet_C "$PC" 120 --no-graph --steps 10 --warmup 3 &&
run lenet_D "$PD" 120 --no-graph --steps 10 --warmup 3 &&
run lenetg_A "$PA" 120 --steps 10 --warmup 3 &&
run rn50_A "$PA" 300 --model resnet50 --steps 2 --warmup 1 &&
run rn50_B "$PB" 300 --model resnet50 --steps 2 --warmup 1 &&
run rn50_C "$PC" 300 --model resnet50 --steps 2 --warmup 1 &&
run vit_A "$PA" 300 --model vit_b16 --steps 2 --warmup 1 &&
run vit_B "$PB" 300 --model vit_b16 --steps 2 --warmup 1
rc=$?
# Reduce on the box (raw counter CSVs of the ResNet/ViT runs exceed gpurun's 64 MiB pull limit).
cd $R
python3 bench/summarize_pmc.py $O/lenet_A $O/lenet_B $O/lenet_C $O/lenet_D --steps 5 --title "LeNet bs1024 fused step (eager launches), PMC" > $O/pmc_lenet.md 2>> $O/summary.txt
python3 bench/summarize_pmc.py $O/lenetg_A --steps 5 --title "LeNet bs1024 fused step (HIP graph), PMC" > $O/pmc_lenet_graph.md 2>> $O/summary.txt
python3 bench/summarize_pmc.py $O/rn50_A $O/rn50_B $O/rn50_C --steps 1 --top 40 --title "ResNet-50 bs256 bf16 step, PMC" > $O/pmc_resnet50.md 2>> $O/summary.txt
python3 bench/summarize_pmc.py $O/vit_A $O/vit_B --steps 1 --top 40 --title "ViT-B/16 bs128 bf16 step, PMC" > $O/pmc_vit_b16.md 2>> $O/summary.txt
for d in $O/*/; do rm -rf "$d"; done
exit $rc
