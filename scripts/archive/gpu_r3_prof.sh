#!/bin/bash
# Round 3: steady-state kernel traces of every model + PMC counter passes (LeNet, ResNet-50, ViT-B/16)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/r3prof; mkdir -p $O
trace() {  # name steps-to-summarise marker args...
  local name=$1 k=$2 mk=$3; shift 3
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$name -o run -- python3 $R/bench.py "$@" > $O/tr_$name.log 2>&1 || return 1
  local f=$(find $O/tr_$name -name '*kernel_trace.csv' | head -1)
  (cd $R && python3 bench/summarize_trace.py "$f" --steps $k --marker $mk --title "$name bf16, 1x MI355X - rocprofv3 --kernel-trace (round 3)") > $O/${name}_kernels.md || return 1
  rm -rf $O/tr_$name
}
trace lenet 50 mlp3_wgrad --steps 200 --warmup 20 &&
trace resnet18 4 _mt_kernel --model resnet18 --steps 6 --warmup 3 &&
trace resnet50 3 _mt_kernel --model resnet50 --steps 5 --warmup 2 &&
trace vit_b16 3 _mt_kernel --model vit_b16 --steps 5 --warmup 2 || exit 1
timeout -s KILL 120 rocprofv3 -L > $O/counters.txt 2>&1 || exit 1
have() { local out=""; for c in "$@"; do grep -qw "$c" $O/counters.txt && out="$out $c"; done; echo $out; }
PA=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT)
PB=$(have SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL)
PC=$(have FETCH_SIZE TCC_HIT_sum)
PD=$(have WRITE_SIZE TCC_MISS_sum TCC_EA0_ATOMIC_sum)
run() {
  local name=$1 ctr=$2; shift 2
  [ -z "$ctr" ] && return 0
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc $ctr -d $O/$name -o run -- python3 $R/bench.py "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> $O/summary.txt; return $rc
}
: > $O/summary.txt
for p in A B C D; do
  eval ctr=\$P$p
  run lenet_$p "$ctr" --steps 40 --warmup 10 && run vit_$p "$ctr" --model vit_b16 --steps 2 --warmup 1 &&
    run rn50_$p "$ctr" --model resnet50 --steps 2 --warmup 1 || exit 1
done
cd $R
python3 bench/summarize_pmc.py $O/lenet_A $O/lenet_B $O/lenet_C $O/lenet_D --steps 5 --top 12 --marker mlp3_wgrad --title "LeNet bs1024 bf16 fused step (round 3: speculative whole-step kernel + weight-gradient/AdamW kernel + batch gather), PMC" > $O/pmc_lenet.md 2>> $O/summary.txt
python3 bench/summarize_pmc.py $O/vit_A $O/vit_B $O/vit_C $O/vit_D --steps 1 --top 30 --title "ViT-B/16 bs128 bf16 step (round 3), PMC" > $O/pmc_vit_b16.md 2>> $O/summary.txt
python3 bench/summarize_pmc.py $O/rn50_A $O/rn50_B $O/rn50_C $O/rn50_D --steps 1 --top 30 --title "ResNet-50 bs256 bf16 step (round 3), PMC" > $O/pmc_resnet50.md 2>> $O/summary.txt
for d in $O/*/; do rm -rf "$d"; done
ls $O
