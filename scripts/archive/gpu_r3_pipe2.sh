#!/bin/bash
# conv tile/pipeline A/B: 8-wave (cfg 0) vs 4-wave 128x128 tiles (cfg 4, 5), outputs checked
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u bench/iconv_probe.py --model resnet50 --cfgs 0,4,5 --check > gpurun_out/pipe2_rn50.jsonl 2> gpurun_out/pipe2_rn50.err || exit 1
timeout -k 10 200 python -u bench/iconv_probe.py --model resnet18 --cfgs 0,4,5 --check > gpurun_out/pipe2_rn18.jsonl 2> gpurun_out/pipe2_rn18.err || exit 1
