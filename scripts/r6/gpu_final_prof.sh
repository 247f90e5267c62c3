#!/bin/bash
# final tree: rocprofv3 kernel-trace stats of the headline LeNet bench (driver shape) and ResNet-18
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6fprof; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lenet -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 \
  > $O/lenet.json 2> $O/lenet.err || { tail -20 $O/lenet.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rn18 -o run -- python3 bench.py --model resnet18 --steps 20 --warmup 5 \
  > $O/rn18.json 2> $O/rn18.err || { tail -20 $O/rn18.err; exit 1; }
find $O -name "*kernel_stats.csv"
