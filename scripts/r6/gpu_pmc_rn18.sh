#!/bin/bash
# ResNet-18 CIFAR PMC (2 SQ passes + memory passes) -> gpurun_out/r6pr/pmc_rn18.md
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6pr; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
C="FETCH_SIZE GRBM_GUI_ACTIVE"
D="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for p in ${PASSES:-A B C D}; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc ${!p} -d $O/w$p -o run -- python3 $R/bench.py --model resnet18 --steps 3 --warmup 2 > $O/w$p.log 2>&1 || { echo "pmc $p failed"; tail -5 $O/w$p.log; exit 1; }
done
cd $R && python3 bench/summarize_pmc.py $(for p in ${PASSES:-A B C D}; do echo $O/w$p; done) --steps 2 --marker sgd_mt_kernel --top 25 --title "ResNet-18 CIFAR bs256 bf16 step (round 6 final), PMC" > $O/pmc_rn18.md
rm -rf $O/wA $O/wB $O/wC $O/wD
cat $O/pmc_rn18.md
