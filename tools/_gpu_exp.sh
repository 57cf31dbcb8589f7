#!/bin/bash
# Quick experiments: bench step pipeline under env knobs.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
run() { # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 1024 > $O/exp_$name.json 2>$O/exp_$name.err || { tail -5 $O/exp_$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/exp_$name.json'));r=d['roofline'];print('$name', round(d['value']/1e9,3),'G', 'pipe_us',round(r['step_pipeline_us'],2),'kern_us',round(r['avg_launch_us'],2))"
}
run base MGX_STAGGER=0
run stag2k MGX_STAGGER=2000
run stag6k MGX_STAGGER=6000
run stag12k MGX_STAGGER=12000
run serial MGX_SERIAL_REFILL=1
