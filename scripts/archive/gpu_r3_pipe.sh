#!/bin/bash
# conv k-tile pipeline A/B (bench/iconv_probe.py, all four configs, outputs checked vs config 0),
# then the round regression
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u bench/iconv_probe.py --model resnet50 --cfgs 0,1,2,3 --check > gpurun_out/pipe_rn50.jsonl 2> gpurun_out/pipe_rn50.err || exit 1
timeout -k 10 200 python -u bench/iconv_probe.py --model resnet18 --cfgs 0,1,2,3 --check > gpurun_out/pipe_rn18.jsonl 2> gpurun_out/pipe_rn18.err || exit 1
bash scripts/gpu_final.sh
