#!/bin/bash
# round 6 box a: DP reduce+AdamW fusion (P2P write-back update) - 2-rank one-GPU tests, W=2 launch
# trace (fused vs unfused), LeNet W=1 driver bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6a; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/gpu/test_ddp_graph.py \
  tests/gpu/test_p2p.py tests/kernels/test_ce_optim.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/lenet_driver.json 2> $O/lenet_driver.err || exit 1
# W=2 on one GPU (gloo host group, P2P transport): each rank under its own rocprofv3
w2() {  # tag, extra env
  local tag=$1; shift
  local port=$((29500 + RANDOM % 1000))
  for r in 0 1; do
    env "$@" MASTER_ADDR=127.0.0.1 MASTER_PORT=$port WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 RANK=$r LOCAL_RANK=$r \
      ROCKET_DIST_BACKEND=gloo ROCKET_P2P=force timeout -k 10 240 rocprofv3 --kernel-trace --stats \
      -d $O/$tag/r$r -o run -- python bench.py --gpus 2 --steps 300 --warmup 20 > $O/${tag}_r$r.json 2> $O/${tag}_r$r.err &
  done
  wait -n || return 1
  wait -n || return 1
}
w2 fused || { tail -20 $O/fused_r0.err; exit 1; }
w2 unfused ROCKET_OPT_EPILOGUE=0 || { tail -20 $O/unfused_r0.err; exit 1; }
for t in fused unfused; do grep -h '"metric"' $O/${t}_r0.json | python3 -c "import json,sys;r=json.loads(sys.stdin.read());print('$t', r['value'], r['ms_per_step'], r['step_ms_p50'], r['dp'].get('transport'), r['dp'].get('capture_mode'), r['dp'].get('replicas_identical'))"; done
python3 -c "import json;r=json.loads(open('$O/lenet_driver.json').read().strip().splitlines()[-1]);print('w1', r['value'], r['ms_per_step'], r['step_ms_p50'], r['host_issue_ms'])"
find $O -name "*kernel_stats.csv" | head
