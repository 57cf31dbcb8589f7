#!/bin/bash
# Builds the diagnostic variants of libmgx.so (switches: csrc/mgx_diag.h) from the current sources, in
# parallel, into ab_libs/libmgx_<name>.so (git-ignored, shipped to the GPU box with the tree while they exist:
# delete them after the A/B -- every gpurun call and the driver's runs push the whole tree).  Usage: bash tools/build_diag_libs.sh [name ...]  (default: all below).
set -e
cd "$(dirname "$0")/../minigrid-rl_amd"
declare -A V=(
  [serial]="-DMGX_SERIAL_REFILL=1"
  [rstamps]="-DMGX_RSTAMPS=1"
  [rstamps_serial]="-DMGX_RSTAMPS=1 -DMGX_SERIAL_REFILL=1"
  [rclock]="-DMGX_REFILL_CLOCK=1 -DMGX_SERIAL_REFILL=1"
  [skip1]="-DMGX_REFILL_CLOCK=1 -DMGX_SERIAL_REFILL=1 -DMGX_GEN_SKIP=1"
  [skip2]="-DMGX_REFILL_CLOCK=1 -DMGX_SERIAL_REFILL=1 -DMGX_GEN_SKIP=2"
  [skip4]="-DMGX_REFILL_CLOCK=1 -DMGX_SERIAL_REFILL=1 -DMGX_GEN_SKIP=4"
  [skip8]="-DMGX_REFILL_CLOCK=1 -DMGX_SERIAL_REFILL=1 -DMGX_GEN_SKIP=8"
  [skip32]="-DMGX_REFILL_CLOCK=1 -DMGX_SERIAL_REFILL=1 -DMGX_GEN_SKIP=32"
  [epw64]="-DMGX_REFILL_EPW=64"
  [epw32]="-DMGX_REFILL_EPW=32"
  [epw16]="-DMGX_REFILL_EPW=16"
  [prio3]="-DMGX_REFILL_PRIO=3"
  [prio1]="-DMGX_REFILL_PRIO=1"
  [prio0]="-DMGX_REFILL_PRIO=0"
  [vmsync]="-DMGX_ROLL_VMKEEP=-1"
  [vm0]="-DMGX_ROLL_VMKEEP=0"
  [vm6]="-DMGX_ROLL_VMKEEP=6"
  [vm4]="-DMGX_ROLL_VMKEEP=4"
  [vm8]="-DMGX_ROLL_VMKEEP=8"
  [vm12]="-DMGX_ROLL_VMKEEP=12"
  [vm16]="-DMGX_ROLL_VMKEEP=16"
  [wg16_serial]="-DMGX_MT_WG1=16 -DMGX_SERIAL_REFILL=1"
  [relaxed]="-DMGX_PUBN_ACQUIRE=0"
  [lprio3]="-DMGX_ROLL_LOGIC_PRIO=3"
  [lprio2]="-DMGX_ROLL_LOGIC_PRIO=2"
  [sfence]="-DMGX_SLIDE_FENCE=1"
  [epb32]="-DMGX_ROLL_EPB_S16=32"
  [slprio3]="-DMGX_STEP_LOGIC_PRIO=3"
  [lp3sf]="-DMGX_ROLL_LOGIC_PRIO=3 -DMGX_SLIDE_FENCE=1"
  [lp3sfrx]="-DMGX_ROLL_LOGIC_PRIO=3 -DMGX_SLIDE_FENCE=1 -DMGX_PUBN_ACQUIRE=0"
  [rclock_np]="-DMGX_REFILL_CLOCK=1"
  [gskip1]="-DMGX_GEN_SKIP=1"
  [gskip2]="-DMGX_GEN_SKIP=2"
  [gskip4]="-DMGX_GEN_SKIP=4"
  [gskip32]="-DMGX_GEN_SKIP=32"
  [prefix2]="-DMGX_GEN_PREFIX2=1"
  [nomemo]="-DMGX_PFX_MEMO=0"
  [lp3p1]="-DMGX_ROLL_LOGIC_PRIO=3 -DMGX_REFILL_PRIO=1"
  [ntrec]="-DMGX_NT_REC=1"
  [ntrows]="-DMGX_NT_ROWS=1"
  [ntboth]="-DMGX_NT_REC=1 -DMGX_NT_ROWS=1"
  [sfence0]="-DMGX_SLIDE_FENCE=0"
  [ntboth_sf0]="-DMGX_NT_REC=1 -DMGX_NT_ROWS=1 -DMGX_SLIDE_FENCE=0"
  [serial_pad4]="-DMGX_SERIAL_REFILL=1 -DMGX_ROLL_LDS_PAD=6000"
  [serial_pad3]="-DMGX_SERIAL_REFILL=1 -DMGX_ROLL_LDS_PAD=13500"
  [pad4]="-DMGX_ROLL_LDS_PAD=6000"
)
names=("$@")
[ ${#names[@]} -eq 0 ] && names=("${!V[@]}")
pids=()
for n in "${names[@]}"; do
  [ -n "${V[$n]+x}" ] || { echo "unknown variant: $n"; exit 1; }
  mkdir -p ../ab_libs
  make -s -B EXTRA="${V[$n]}" OUT=../ab_libs/libmgx_$n.so > /tmp/build_diag_$n.log 2>&1 &
  pids+=($!)
  while [ $(jobs -rp | wc -l) -ge 4 ]; do sleep 1; done
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
[ $rc -eq 0 ] || { echo "a diag build failed: /tmp/build_diag_*.log"; exit 1; }
echo "built: ${names[*]}"
