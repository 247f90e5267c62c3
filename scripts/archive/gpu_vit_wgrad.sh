#!/bin/bash
# ViT-B/16 library-GEMM parameter-gradient path: tests, then the bench with bf16 / fp32 split-K
# partials (ROCKET_WGRAD_F32), then a kernel trace of the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; : > gpurun_out/vit_wgrad.jsonl; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/kernels/test_mgemm.py tests/kernels/test_linear_conv.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/test_mgemm.log 2>&1
rc=$?; tail -3 gpurun_out/test_mgemm.log; [ $rc -eq 0 ] || exit $rc
for f32 in 0 1 0; do
  ROCKET_WGRAD_F32=$f32 timeout -k 10 300 python bench.py --model vit_b16 --steps 10 --warmup 3 2> gpurun_out/vit_f$f32.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'wgrad_f32':$f32,'value':d['value'],'ms':d['ms_per_step'],'p50':d['step_ms_p50'],'host':d['host_ms_p50']}))" >> gpurun_out/vit_wgrad.jsonl || exit 1
done
cat gpurun_out/vit_wgrad.jsonl
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_vit -o run -- python3 $R/bench.py --model vit_b16 --steps 5 --warmup 2 > $R/gpurun_out/prof_vit.log 2>&1 || exit 1
cd $R && f=$(find gpurun_out/prof_vit -name '*kernel_trace.csv' | head -1) && python3 bench/summarize_trace.py "$f" --steps 4 --title "ViT-B/16 224^2 bf16 bs128, 1x MI355X - rocprofv3 --kernel-trace" > gpurun_out/vit_kernels.md; rc=$?
rm -rf gpurun_out/prof_vit
exit $rc
