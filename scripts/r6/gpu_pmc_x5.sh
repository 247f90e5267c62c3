#!/bin/bash
# PMC passes over single GEMM runs (x5 / x4 / lib) -> gpurun_out/r6pmc/*.md
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6pmc; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
PB="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
for case in ${CASES:-sq8192:x5 sq8192:lib qkv:x5 qkv:lib}; do
  shp=${case%%:*}; eng=${case##*:}
  for p in A B; do
    eval ctr=\$P$p
    timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $ctr -d $O/${shp}_${eng}_$p -o run -- python3 $R/bench/x5_one.py $shp $eng 4 > $O/${shp}_${eng}_$p.log 2>&1 || { echo "pass $case $p failed"; tail -5 $O/${shp}_${eng}_$p.log; exit 1; }
  done
  cd $R && python3 bench/summarize_pmc.py $O/${shp}_${eng}_A $O/${shp}_${eng}_B --steps 1 --marker __none__ --top 4 --title "$shp $eng" > $O/${shp}_${eng}.md 2>&1; cd /tmp
  rm -rf $O/${shp}_${eng}_A $O/${shp}_${eng}_B
done
cat $O/*.md | grep -v "^$" | cut -c1-400
