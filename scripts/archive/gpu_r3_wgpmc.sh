#!/bin/bash
# wgrad vs fwd of one ResNet-18 conv shape (Cin 128, 16x16, 3x3): kernel trace + 2 PMC passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/wgpmc; mkdir -p $O
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench/iconv_probe.py --model resnet18 --only c128h16k3s1,c64h32k3s1 --dirs fwd,wgrad > $O/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $A -d $O/pA -o run -- python3 $R/bench/iconv_probe.py --model resnet18 --only c128h16k3s1 --dirs fwd,wgrad > $O/pA.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $B -d $O/pB -o run -- python3 $R/bench/iconv_probe.py --model resnet18 --only c128h16k3s1 --dirs fwd,wgrad > $O/pB.log 2>&1 || exit 1
cd $R
python3 bench/summarize_pmc.py $O/pA $O/pB --marker NO_MARKER --steps 1 --top 10 --title "ResNet-18 conv c128 16x16 3x3: fwd vs wgrad, PMC" > $O/pmc.md 2>&1
cat $O/pmc.md
find $O/trace -name "*kernel_stats.csv" -exec cat {} \;
