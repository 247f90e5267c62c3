#!/bin/bash
# round 5: kernel-argument placement (HIP_FORCE_DEV_KERNARG unset / 1 / 0) on the LeNet step:
# driver-shape and long benches alternating, then a phase timeline per setting
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ka; rm -rf $O; mkdir -p $O
cd $R && export TMPDIR=/tmp
for pass in 1 2; do
  for v in def k1 k0; do
    unset HIP_FORCE_DEV_KERNARG
    [ $v = k1 ] && export HIP_FORCE_DEV_KERNARG=1
    [ $v = k0 ] && export HIP_FORCE_DEV_KERNARG=0
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_${v}_$pass.json 2>> $O/err.log || exit 1
    timeout -k 10 120 python bench.py --steps 1000 --warmup 50 > $O/long_${v}_$pass.json 2>> $O/err.log || exit 1
    for f in drv_${v}_$pass long_${v}_$pass; do python3 -c "import json;r=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', r['value'], r['ms_per_step'], r['step_ms_p50'], r.get('host_issue_ms'))"; done
  done
done
for v in def k1 k0; do
  unset HIP_FORCE_DEV_KERNARG
  [ $v = k1 ] && export HIP_FORCE_DEV_KERNARG=1
  [ $v = k0 ] && export HIP_FORCE_DEV_KERNARG=0
  ROCKET_LENET_TRACE=$O/tl_$v.json timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $O/tl_$v.out 2>>$O/err.log || exit 1
  python3 -c "
import json; d=json.load(open('$O/tl_$v.json')); s=d['spans']; g=s['wgrad_groups']['fc1 tiles']
print('$v', json.dumps({k: s[k] for k in ('fwd','bwd')}), 'wgrad', s['wgrad']['first_start'], g['median_old_loaded'], s['wgrad']['median_end'])"
done
