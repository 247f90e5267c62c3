#!/bin/bash
# HIP runtime knobs vs. graph replay cost: graph probe + LeNet bench under each setting.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
S=gpurun_out/summary_env.txt
: > $S
run() {
  name=$1; shift
  env "$@" timeout -k 10 120 python bench/graph_launch_probe.py > gpurun_out/env_probe_$name.json 2> gpurun_out/env_probe_$name.err || { echo "$name probe FAILED" >> $S; exit 1; }
  env "$@" timeout -k 10 180 python bench.py --steps 400 --warmup 40 > gpurun_out/env_bench_$name.json 2> gpurun_out/env_bench_$name.err || { echo "$name bench FAILED" >> $S; exit 1; }
  echo "$name $(cat gpurun_out/env_probe_$name.json) $(python -c "import json;d=json.load(open('gpurun_out/env_bench_$name.json'));print(d['value'],d['ms_per_step'],d['host_ms_p50'])")" >> $S
}
run base X=1
run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run devkarg1 HIP_FORCE_DEV_KERNARG=1
run devkarg0 HIP_FORCE_DEV_KERNARG=0
run hdpwa0 DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0
run batch64 DEBUG_HIP_GRAPH_BATCH_SIZE=64
run graphq0 DEBUG_HIP_FORCE_GRAPH_QUEUES=0
run kcopy0 DEBUG_HIP_KERNARG_COPY_OPT=0
run skipkarg1 ROC_SKIP_KERNEL_ARG_COPY=1
exit 0
