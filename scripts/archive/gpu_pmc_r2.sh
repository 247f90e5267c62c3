#!/bin/bash
# Round-2 PMC refresh: ResNet-50 (4 passes) and ViT-B/16 (2 passes) with the current kernels, plus
# an fp16 (GradScaler) ResNet-18 kernel trace checked for torch's unscale kernel.
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
run() {
  local name=$1 ctr=$2 to=$3; shift 3
  [ -z "$ctr" ] && return 0
  timeout -s KILL $to rocprofv3 --kernel-trace --output-format csv --pmc $ctr -d $O/$name -o run -- python3 $R/bench.py "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> $O/summary.txt; return $rc
}
: > $O/summary.txt
run rn50_A "$PA" 300 --model resnet50 --steps 2 --warmup 1 &&
run rn50_B "$PB" 300 --model resnet50 --steps 2 --warmup 1 &&
run rn50_C "$PC" 300 --model resnet50 --steps 2 --warmup 1 &&
run rn50_D "$PD" 300 --model resnet50 --steps 2 --warmup 1 &&
run vit_A "$PA" 300 --model vit_b16 --steps 2 --warmup 1 &&
run vit_B "$PB" 300 --model vit_b16 --steps 2 --warmup 1
rc=$?
cd $R
python3 bench/summarize_pmc.py $O/rn50_A $O/rn50_B $O/rn50_C $O/rn50_D --steps 1 --top 40 --title "ResNet-50 bs256 bf16 step (round 2 kernels), PMC" > $O/pmc_resnet50.md 2>> $O/summary.txt
python3 bench/summarize_pmc.py $O/vit_A $O/vit_B --steps 1 --top 40 --title "ViT-B/16 bs128 bf16 step (round 2 kernels), PMC" > $O/pmc_vit_b16.md 2>> $O/summary.txt
for d in $O/*/; do rm -rf "$d"; done
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_fp16 -o run -- python3 $R/bench.py --model resnet18 --mp fp16 --steps 5 --warmup 2 > $R/gpurun_out/prof_fp16.log 2>&1 || exit 1
cd $R && f=$(find gpurun_out/prof_fp16 -name '*kernel_trace.csv' | head -1) && python3 bench/summarize_trace.py "$f" --steps 3 --title "ResNet-18 fp16 (device GradScaler) - rocprofv3 --kernel-trace" > gpurun_out/kernels_resnet18_fp16.md
echo "unscale kernels in the whole fp16 trace: $(grep -c "non_finite_check_and_unscale" $f)" >> gpurun_out/kernels_resnet18_fp16.md
rm -rf gpurun_out/prof_fp16
