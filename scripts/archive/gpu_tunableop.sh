#!/bin/bash
# ViT-B/16 GEMM selection: tune the K-split weight-gradient (strided-batched) shapes with TunableOp
# into gpurun_out/tunableop_split.csv, then measure with the merged table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/summary_tunable.txt
: > $S
ROCKET_TUNE_GEMMS=1 ROCKET_TUNED_GEMMS_OUT=$R/gpurun_out/tunableop_split.csv \
  timeout -k 10 700 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/vit_split_tune.json 2> gpurun_out/vit_split_tune.err; echo "tune rc=$?" >> $S
timeout -k 10 400 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/vit_split_table.json 2> gpurun_out/vit_split_table.err; echo "split(shipped table) rc=$?" >> $S
exit 0
