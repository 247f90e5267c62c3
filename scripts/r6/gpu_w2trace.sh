#!/bin/bash
# LeNet W=2 (two ranks on one GPU, P2P transport, fused reduce+AdamW) launch trace -> small summaries
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6w2; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
port=$((29500 + RANDOM % 1000))
for r in 0 1; do
  env ${EXTRA_ENV} MASTER_ADDR=127.0.0.1 MASTER_PORT=$port WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 RANK=$r LOCAL_RANK=$r \
    ROCKET_DIST_BACKEND=gloo ROCKET_P2P=force timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
    -d $O/t/r$r -o run -- python bench.py --gpus 2 --steps 100 --warmup 20 > $O/r$r.json 2> $O/r$r.err &
done
wait -n || { tail -20 $O/r0.err; exit 1; }
wait -n || { tail -20 $O/r1.err; exit 1; }
for r in 0 1; do
python3 - $O/t/r$r $r > $O/summary_r$r.txt <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# steady state: the last 50 occurrences of the step's first kernel mark steps
names = [r["Kernel_Name"] for r in rows]
first = names[-1]
# step = sequence between consecutive launches of the whole-step kernel
idx = [i for i, n in enumerate(names) if "lenet_train_kernel" in n]
print(f"rank {sys.argv[2]}: {len(rows)} kernels traced, {len(idx)} whole-step launches")
a, b = idx[-2], idx[-1]
print("one steady step (launch order, us, start offset from the step's first kernel):")
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3; d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"  +{s:7.2f}  {d:6.2f} us  grid {r.get('Grid_Size',''):>7}  {r['Kernel_Name'][:90]}")
per = collections.defaultdict(list)
for r in rows[idx[-51]:idx[-1]]:
    per[r["Kernel_Name"][:90]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print("last 50 steps: launches per step and mean us")
for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {len(v)/50:5.2f}/step  {sum(v)/len(v):7.2f} us  {n}")
PY
done
rm -rf $O/t
grep -h '"metric"' $O/r0.json | python3 -c "import json,sys;r=json.loads(sys.stdin.read());print('w2', r['value'], r['ms_per_step'], r.get('step_ms_p50'), r['dp'].get('transport'), r['dp'].get('capture_mode'))"
cat $O/summary_r0.txt
