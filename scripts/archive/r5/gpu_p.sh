#!/bin/bash
# round 5 box p: host-path trims (StepLR fast path, cached hyperparameter check, version token): graph /
# optimizer / scheduler tests, LeNet driver + long bench (host_issue_ms)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-r5p}; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_graph_capture.py \
  tests/kernels/test_ce_optim.py tests/kernels/test_amp.py tests/gpu/test_launcher_gpu.py tests/examples > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.json 2>> $O/err.log || exit 1
  timeout -k 10 120 python bench.py --steps 1000 --warmup 50 > $O/long_$i.json 2>> $O/err.log || exit 1
  for f in drv_$i long_$i; do python3 -c "import json;r=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', r['value'], r['ms_per_step'], r['step_ms_p50'], 'host_issue', r['host_issue_ms'], 'host_p50', r['host_ms_p50'])"; done
done
timeout -k 10 120 python bench.py --mp fp16 --steps 1000 --warmup 50 > $O/fp16.json 2>> $O/err.log || exit 1
python3 -c "import json;r=json.loads(open('$O/fp16.json').read().strip().splitlines()[-1]);print('fp16', r['value'], r['ms_per_step'], 'host_issue', r['host_issue_ms'])"
