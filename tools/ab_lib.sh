#!/bin/bash
# A/B of two library builds on one box: the C3 bench alternating XTRL_LIB=<base .so> and the
# in-tree build, N rounds each (box-to-box variation is larger than most single changes).
# Usage: tools/ab_lib.sh ab/libxtrl_base.so [rounds]
set -u
mkdir -p gpurun_out
base=$1; rounds=${2:-2}
for r in $(seq $rounds); do
  for arm in base new; do
    if [ $arm = base ]; then lib=$base; else lib=x-transformers-rl_amd/xtrl_amd/libxtrl_hip.so; fi
    XTRL_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/ab_$arm.log 2>&1 || exit 1
    echo -n "$arm: "; tail -1 gpurun_out/ab_$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phase_ms'])"
  done
done
