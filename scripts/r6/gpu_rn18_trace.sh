#!/bin/bash
# ResNet-18 CIFAR step: kernels per step, summed kernel time vs wall -> gpurun_out/r6rn/rn18.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6rn; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 $R/bench.py --model ${MODEL:-resnet18} --steps 6 --warmup 3 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
python3 - $O/t > $O/rn18.txt <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "_mt_kernel" in r["Kernel_Name"]]  # optimizer launch ends a step
a, b = idx[-4], idx[-1]
seg = rows[a + 1: b + 1]
steps = 3
wall = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3 / steps
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3 / steps
print(f"kernels/step {len(seg)/steps:.0f}  wall/step {wall:.1f} us  summed kernel time/step {busy:.1f} us  idle {wall-busy:.1f} us")
c = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:90]
    c[n][0] += 1; c[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for n, (k, t) in sorted(c.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"{k/steps:6.1f}/step {t/steps:9.1f} us  {n}")
with open(sys.argv[1] + "/../seq.txt", "w") as fo:  # the last step's launch sequence
    for r in rows[idx[-2] + 1: idx[-1] + 1]:
        fo.write(f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.1f}  {r['Kernel_Name'][:110]}\n")
PY
rm -rf $O/t
cat $O/rn18.txt
