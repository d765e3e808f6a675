#!/bin/bash
# A/B of two library builds on one box: the C3 bench alternating XTRL_LIB=<base .so> and the
# in-tree build, N rounds each (box-to-box variation is larger than most single changes).
# Usage: tools/ab_lib.sh ab/libxtrl_base.so [rounds] [config]  (the new arm: XTRL_NEW or the in-tree build)
set -u
mkdir -p gpurun_out
base=$1; rounds=${2:-2}; cfg=${3:-c3}; new=${XTRL_NEW:-x-transformers-rl_amd/xtrl_amd/libxtrl_hip.so}
for r in $(seq $rounds); do
  for arm in base new; do
    if [ $arm = base ]; then lib=$base; else lib=$new; fi
    XTRL_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/ab_$arm.log 2>&1 || exit 1
    echo -n "$arm: "; tail -1 gpurun_out/ab_$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phase_ms'])"
  done
done
