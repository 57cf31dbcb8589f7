#!/bin/bash
# One gpurun call: bench each diagnostic build given as "name[:ENV=VAL]" (libmgx_<name>.so;
# "cur" = libmgx.so).  Bench only; every step has its own time limit.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; env=""; [ "$spec" != "$name" ] && env=${spec#*:}
  lib=$R/minigrid-rl_amd/mgx/libmgx_$name.so; [ "$name" = cur ] && lib=$R/minigrid-rl_amd/mgx/libmgx.so
  tag=$(echo "$spec" | tr ':=' '__')
  env MGX_LIB_PATH=$lib $env timeout -k 10 200 python bench.py --steps 1024 --warmup 64 --cpu-seconds 0 --probe 128 > gpurun_out/var_$tag.json 2>gpurun_out/var_$tag.err
  python3 -c "import json; d=json.load(open('gpurun_out/var_$tag.json')); r=d['roofline']; print('%-28s %.3f G/s %6.2f us/step kernel %6.2f us' % ('$spec', d['value']/1e9, d['ms_per_step']*1e3, r['avg_launch_us']))"
done
