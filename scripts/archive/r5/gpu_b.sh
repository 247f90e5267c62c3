#!/bin/bash
# round 5 box b: x4 GEMM phase stamps; PMC passes with HBM/L2 counters (LeNet, ResNet-50, ViT-B/16);
# kernel traces at HEAD (ViT-B/16 fp16, ResNet-50 bf16)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5b; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 200 python bench/x4_trace.py --out $O/x4_trace.json > $O/x4_trace.log 2>&1 || { tail -20 $O/x4_trace.log; exit 1; }
cat $O/x4_trace.log
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || exit 1
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
C="FETCH_SIZE GRBM_GUI_ACTIVE"
D="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
pmc() {  # name counters cmd...
  local n=$1 c=$2; shift 2
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc $c -d $O/$n -o run -- "$@" > $O/$n.log 2>&1
}
for p in A B C D; do pmc l$p "${!p}" python3 $R/bench.py --steps 30 --warmup 10 || { echo "lenet pmc $p failed"; tail -5 $O/l$p.log; exit 1; }; done
cd $R && python3 bench/summarize_pmc.py $O/lA $O/lB $O/lC $O/lD --steps 10 --marker mlp3_wgrad_kernel --title "LeNet bs1024 captured step (launch-list replay), PMC, round 5" > gpurun_out/r5_pmc_lenet_progression.md
cd /tmp
for p in A B C D; do pmc r$p "${!p}" python3 $R/bench.py --model resnet50 --steps 3 --warmup 2 || { echo "resnet pmc $p failed"; tail -5 $O/r$p.log; exit 1; }; done
cd $R && python3 bench/summarize_pmc.py $O/rA $O/rB $O/rC $O/rD --steps 2 --marker sgd_mt_kernel --top 25 --title "ResNet-50 bs256 bf16 captured step, PMC, round 5" > gpurun_out/r5_pmc_resnet50.md
cd /tmp
for p in A B C D; do pmc v$p "${!p}" python3 $R/bench.py --model vit_b16 --steps 3 --warmup 2 || { echo "vit pmc $p failed"; tail -5 $O/v$p.log; exit 1; }; done
cd $R && python3 bench/summarize_pmc.py $O/vA $O/vB $O/vC $O/vD --steps 2 --marker adam_mt_kernel --top 25 --title "ViT-B/16 bs128 bf16 captured step, PMC, round 5" > gpurun_out/r5_pmc_vit_b16.md
for d in lA lB lC lD rA rB rC rD vA vB vC vD; do rm -rf $O/$d; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/vf16 -o run -- python3 $R/bench.py --model vit_b16 --mp fp16 --steps 8 --warmup 3 > $O/vf16.log 2>&1 || { tail -20 $O/vf16.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/r50 -o run -- python3 $R/bench.py --model resnet50 --steps 8 --warmup 3 > $O/r50.log 2>&1 || { tail -20 $O/r50.log; exit 1; }
cd $R
f=$(find $O/vf16 -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 5 --title "ViT-B/16 bs128 fp16 step (round 5, HEAD), rocprofv3 kernel trace" > gpurun_out/r5_vit_b16_fp16_kernels.md
f=$(find $O/r50 -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 5 --marker sgd_mt_kernel --title "ResNet-50 bs256 bf16 step (round 5, HEAD), rocprofv3 kernel trace" > gpurun_out/r5_resnet50_kernels.md
rm -rf $O/vf16 $O/r50
head -16 gpurun_out/r5_pmc_lenet_progression.md gpurun_out/r5_pmc_vit_b16.md
