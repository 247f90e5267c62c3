#!/bin/bash
# ViT-B/16 with PyTorch TunableOp GEMM selection (hipBLASLt + rocBLAS solutions benchmarked at
# first use) vs the default heuristics; the tuned table is written to gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/summary_tunable.txt
: > $S
timeout -k 10 400 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/vit_default.json 2> gpurun_out/vit_default.err; echo "default rc=$?" >> $S
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_vit%d.csv \
  timeout -k 10 700 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/vit_tune.json 2> gpurun_out/vit_tune.err; echo "tune rc=$?" >> $S
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_vit%d.csv \
  timeout -k 10 400 python bench.py --model vit_b16 --steps 20 --warmup 5 > gpurun_out/vit_tuned.json 2> gpurun_out/vit_tuned.err; echo "tuned rc=$?" >> $S
exit 0
