#!/bin/bash
# round 5 box e: x4 fused MLP epilogues (GELU fwd, gelu'+colsum dgrad) - kernel tests, ViT bench A/B
# (ROCKET_VIT_X4_MLP=1 vs 0, interleaved), ViT kernel trace with the fusions
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5e; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_xgemm4.py \
  tests/kernels/test_mgemm.py tests/kernels/test_fp16_vit.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0 1 0; do
  ROCKET_VIT_X4_MLP=$v timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 > $O/vit_$v.json 2>> $O/err.log || exit 1
  python3 -c "import json;r=json.loads(open('$O/vit_$v.json').read().strip().splitlines()[-1]);print('x4_mlp=$v', r['value'], r['ms_per_step'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/vit -o run -- python3 $R/bench.py --model vit_b16 --steps 8 --warmup 3 > $O/vit_trace.log 2>&1 || { tail -20 $O/vit_trace.log; exit 1; }
cd $R
f=$(find $O/vit -name "*kernel_trace.csv" | head -1)
python3 bench/summarize_trace.py $f --steps 5 --title "ViT-B/16 bs128 bf16 step (round 5, fused x4 MLP GEMMs), rocprofv3 kernel trace" > gpurun_out/r5_vit_b16_kernels.md
rm -rf $O/vit
head -30 gpurun_out/r5_vit_b16_kernels.md
