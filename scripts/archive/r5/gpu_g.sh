#!/bin/bash
# round 5 box g: LeNet step timeline with per-wave stamps (forward conv1 / conv2, backward phase B) +
# PMC passes (LDS bank conflicts, MFMA, HBM / L2) of the current LeNet kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5g; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_linear_conv.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ROCKET_LENET_TRACE=$O/timeline.json timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $O/tl.json 2>>$O/err.log || exit 1
python3 -c "
import json; d=json.load(open('$O/timeline.json'))
for k,v in d['waves'].items(): print(k, v)
for p in d['fwd_phases']+d['bwd_phases']: print(p['phase'], p['median_us_since_prev'])"
cd /tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
C="FETCH_SIZE GRBM_GUI_ACTIVE"
D="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for p in A B C D; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc ${!p} -d $O/l$p -o run -- python3 $R/bench.py --steps 30 --warmup 10 > $O/l$p.log 2>&1 || { echo "lenet pmc $p failed"; tail -5 $O/l$p.log; exit 1; }
done
cd $R && python3 bench/summarize_pmc.py $O/lA $O/lB $O/lC $O/lD --steps 10 --marker mlp3_wgrad_kernel --title "LeNet bs1024 captured step (launch-list replay), PMC, round 5 (KeepSmem forward state, LDS-DMA wgrad)" > gpurun_out/r5_pmc_lenet_progression.md
rm -rf $O/lA $O/lB $O/lC $O/lD
cat gpurun_out/r5_pmc_lenet_progression.md
