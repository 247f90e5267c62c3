#!/bin/bash
# Round-4 PMC passes (own runs, --kernel-trace + --pmc only): captured LeNet step, ResNet-50, ViT-B/16
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/r4pmc; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 -L > $O/counters.txt 2>&1 || exit 1
have() { local out=""; for c in "$@"; do grep -qw "$c" $O/counters.txt && out="$out $c"; done; echo $out; }
A=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE)
B=$(have SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE)
echo "A: $A / B: $B" > $O/passes.txt
pmc() {  # name counters cmd...
  local n=$1 c=$2; shift 2
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc $c -d $O/$n -o run -- "$@" > $O/$n.log 2>&1
}
pmc lA "$A" python3 $R/bench.py --steps 30 --warmup 10 &&
pmc lB "$B" python3 $R/bench.py --steps 30 --warmup 10 || { echo "lenet pmc failed"; tail -5 $O/lA.log $O/lB.log; exit 1; }
cd $R && python3 bench/summarize_pmc.py $O/lA $O/lB --steps 10 --marker mlp3_wgrad_kernel --title "LeNet bs1024 captured step (launch-list replay), PMC, round 4" > gpurun_out/r4_pmc_lenet.md
cd /tmp
pmc rA "$A" python3 $R/bench.py --model resnet50 --steps 3 --warmup 2 &&
pmc rB "$B" python3 $R/bench.py --model resnet50 --steps 3 --warmup 2 || { echo "resnet pmc failed"; exit 1; }
cd $R && python3 bench/summarize_pmc.py $O/rA $O/rB --steps 2 --marker sgd_mt_kernel --top 25 --title "ResNet-50 bs256 bf16 captured step, PMC, round 4" > gpurun_out/r4_pmc_resnet50.md
cd /tmp
pmc vA "$A" python3 $R/bench.py --model vit_b16 --steps 3 --warmup 2 &&
pmc vB "$B" python3 $R/bench.py --model vit_b16 --steps 3 --warmup 2 || { echo "vit pmc failed"; exit 1; }
cd $R && python3 bench/summarize_pmc.py $O/vA $O/vB --steps 2 --marker adam_mt_kernel --top 25 --title "ViT-B/16 bs128 bf16 captured step, PMC, round 4" > gpurun_out/r4_pmc_vit_b16.md
for d in lA lB rA rB vA vB; do rm -rf $O/$d; done
head -12 gpurun_out/r4_pmc_lenet.md; head -14 gpurun_out/r4_pmc_resnet50.md; head -14 gpurun_out/r4_pmc_vit_b16.md
