#!/bin/bash
# Repeat of the packet-capture A/B plus a host-side cProfile of the LeNet bench loop.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
S=gpurun_out/summary_env2.txt
: > $S
run() {
  name=$1; shift
  env "$@" timeout -k 10 180 python bench.py --steps 1000 --warmup 50 > gpurun_out/env2_$name.json 2> gpurun_out/env2_$name.err || { echo "$name bench FAILED" >> $S; exit 1; }
  echo "$name $(python -c "import json;d=json.load(open('gpurun_out/env2_$name.json'));print(d['value'],d['ms_per_step'],d['step_ms_p50'],d['host_ms_p50'])")" >> $S
}
for i in 1 2; do
  run base$i X=1
  run pktcap0_$i DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run pk0dk1_$i DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 HIP_FORCE_DEV_KERNARG=1
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 180 python -m cProfile -o gpurun_out/host.prof bench.py --steps 2000 --warmup 50 > gpurun_out/env2_prof.json 2>&1 || { echo "prof FAILED" >> $S; exit 1; }
python - <<'PY' > gpurun_out/host_prof.txt
import pstats
p = pstats.Stats("gpurun_out/host.prof")
p.sort_stats("tottime").print_stats(45)
PY
rm -f gpurun_out/host.prof
exit 0
