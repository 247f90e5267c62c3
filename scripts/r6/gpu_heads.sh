#!/bin/bash
# native classifier heads: mgemm tests, ResNet-50 / ViT benches and a ResNet-50 trace check for library GEMMs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6h; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_mgemm.py -k "mixed or small_head" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
VARIANTS="rn50:ROCKET_VIT_GEMM=mixed vit:ROCKET_VIT_GEMM=mixed" true
timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/rn50.json 2> $O/rn50.err || { tail -20 $O/rn50.err; exit 1; }
python3 -c "import json;r=json.loads(open('$O/rn50.json').read().strip().splitlines()[-1]);print('resnet50', r['value'])"
timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/rn18.json 2> $O/rn18.err || { tail -20 $O/rn18.err; exit 1; }
python3 -c "import json;r=json.loads(open('$O/rn18.json').read().strip().splitlines()[-1]);print('resnet18', r['value'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 $R/bench.py --model resnet50 --steps 3 --warmup 2 > $O/tr.log 2>&1 || { tail -20 $O/tr.log; exit 1; }
python3 - $O/tr <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
lib = [r for r in rows if "Cijk" in r["Name"]]
print("resnet50 trace: kernels", len(rows), "library GEMM kernels", len(lib), [r["Name"][:60] for r in lib])
PY
rm -rf $O/tr
