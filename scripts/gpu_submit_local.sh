#!/bin/bash
# usage: gpu_submit.sh <outfile> <timeout> <script>  -- resubmits only when gpurun reports nothing ran
out=$1; to=$2; shift 2
for i in 1 2 3 4 5 6; do
  timeout $((to + 1500)) /usr/local/graft/bin/gpurun --timeout $to -- "$@" > "$out" 2>&1
  if grep -q "status=transient" "$out" && grep -qE "charged=(0.0s|Nones)" "$out"; then sleep 90; continue; fi
  break
done
