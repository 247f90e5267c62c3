#!/bin/bash
# xgemm probe: numerics + speed vs hipBLASLt and rk_mgemm tile 0 (args passed to the probe)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u bench/xgemm_probe.py "$@" > gpurun_out/xgemm_probe.log 2>&1; rc=$?
python3 - <<'PY'
import json
for l in open("gpurun_out/xgemm_probe.jsonl"):
    r = json.loads(l)
    cells = " ".join(f"{k}={v.get('tflops','-')}/{v.get('rel_err','E')}" for k, v in r.items() if isinstance(v, dict))
    print(r["case"], r["dir"], "best", r["best"], r["best_vs_lib"], "|", cells)
PY
exit $rc
