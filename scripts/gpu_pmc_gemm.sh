#!/bin/bash
# PMC passes over the native GEMM at ViT shapes (bench/mgemm_one.py); summary -> gpurun_out/pmc_gemm/pmc_mgemm.md
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmc_gemm; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 -L > $O/counters.txt 2>&1 || exit 1
have() { local out=""; for c in "$@"; do grep -qw "$c" $O/counters.txt && out="$out $c"; done; echo $out; }
PA=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE)
PB=$(have SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE)
PC=$(have TCC_HIT_sum TCC_MISS_sum TCC_BUSY_sum GRBM_GUI_ACTIVE)
PD=$(have FETCH_SIZE GRBM_GUI_ACTIVE)
echo "A: $PA / B: $PB / C: $PC / D: $PD" > $O/passes.txt
CASES="$@"
for p in A B C D; do
  eval ctr=\$P$p
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $ctr -d $O/$p -o run -- python3 $R/bench/mgemm_one.py $CASES > $O/$p.log 2>&1 || { echo "pass $p failed" >> $O/passes.txt; exit 1; }
done
cd $R && python3 bench/summarize_pmc.py $O/A $O/B $O/C $O/D --steps 1 --marker __none__ --top 30 --title "rk_mgemm at ViT-B/16 shapes, PMC" > $O/pmc_mgemm.md
for d in $O/A $O/B $O/C $O/D; do rm -rf "$d"; done
