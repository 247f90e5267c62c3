#!/bin/bash
# xgemm5 timing ablations (build_abl/abl<n>, scripts/r6/build_x5_abl.sh): probe each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6abl; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
for n in base ${ABL:-$(ls $R/build_abl)}; do
  D=$R/rocket_amd/_lib; [ $n != base ] && D=$R/build_abl/$n
  ROCKET_LIBDIR=$D timeout -k 10 200 python bench/gemm_r6_probe.py --out $O/p$n.jsonl --rounds 2 --shapes ${SHAPES:-sq8192,fc1,proj} > $O/p$n.log 2>&1 || { tail -20 $O/p$n.log; exit 1; }
  python3 - $O/p$n.jsonl $n <<'PY'
import json,sys
for l in open(sys.argv[1]):
    r=json.loads(l); print('abl', sys.argv[2], r['case'], 'lib', r['lib']['tflops'], 'x5', r['x5']['tflops'], 'w4', r['x5_256x256']['tflops'], r['x5_128x256']['tflops'], r['x5_256x128']['tflops'], 'w8', r['w8_256x256']['tflops'], r['w8_128x256']['tflops'], r['w8_256x128']['tflops'])
PY
done
