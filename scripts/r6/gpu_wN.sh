#!/bin/bash
# LeNet bench.py with W ranks sharing one GPU (gloo host group, P2P transport): a rehearsal of the
# W-rank data-parallel step (correctness / launch structure, not throughput)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
W=${W:-4}
O=$R/gpurun_out/r6w$W; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
port=$((29500 + RANDOM % 1000))
for r in $(seq 0 $((W - 1))); do
  MASTER_ADDR=127.0.0.1 MASTER_PORT=$port WORLD_SIZE=$W LOCAL_WORLD_SIZE=$W RANK=$r LOCAL_RANK=$r \
    ROCKET_DIST_BACKEND=gloo ROCKET_P2P=force timeout -k 10 240 python bench.py --gpus $W --steps 60 --warmup 10 \
    > $O/r$r.json 2> $O/r$r.err &
done
for r in $(seq 0 $((W - 1))); do wait -n || { tail -20 $O/r0.err; exit 1; }; done
grep -h '"metric"' $O/r0.json | python3 -c "import json,sys;r=json.loads(sys.stdin.read());print('W', r['n_gpus'], r['value'], r['ms_per_step'], r['dp'])"
