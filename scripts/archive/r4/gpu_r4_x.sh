#!/bin/bash
# xgemm evaluation batch: isolated probe, kernel tests, ViT routes (bf16 lib vs x, fp16 x)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
S=gpurun_out/r4x_summary.txt; : > $S
timeout -k 10 300 python -u bench/xgemm_probe.py --cfgs 0,20,21 --splits 1,4,9 > gpurun_out/xgemm_probe.log 2>&1 || { echo "probe rc=$?" >> $S; exit 1; }
python3 - >> $S <<'PY'
import json
for l in open("gpurun_out/xgemm_probe.jsonl"):
    r = json.loads(l)
    cells = " ".join(f"{k}={v.get('tflops','-')}/{v.get('rel_err','E')}" for k, v in r.items() if isinstance(v, dict))
    print(r["case"], r["dir"], "best", r["best"], r["best_vs_lib"], "|", cells)
PY
timeout -k 10 400 python -u -m pytest tests/kernels/test_xgemm.py tests/kernels/test_fp16_vit.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r4x_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $S; tail -3 gpurun_out/r4x_pytest.log >> $S
[ $rc -le 1 ] || exit $rc
for cfg in "lib bf16" "x bf16" "x fp16"; do
  set -- $cfg
  ROCKET_VIT_GEMM=$1 timeout -k 10 300 python bench.py --model vit_b16 --steps 20 --warmup 5 --mp $2 > gpurun_out/r4x_vit_$1_$2.json 2> gpurun_out/r4x_vit_$1_$2.err || { echo "vit $1 $2 failed" >> $S; tail -5 gpurun_out/r4x_vit_$1_$2.err >> $S; exit 1; }
  python3 -c "import json;r=json.load(open('gpurun_out/r4x_vit_$1_$2.json'));print('vit $1 $2', r['value'], r['ms_per_step'])" >> $S
done
cat $S
