#!/bin/bash
# A/B/C: a saved worktree (base), this tree, and this tree under an environment switch ("VAR=value"),
# alternating, N rounds.  Usage: tools/ab_env.sh <base dir> <VAR=value> [rounds] [config]
set -u
mkdir -p gpurun_out
base=$1; envsw=$2; rounds=${3:-2}; cfg=${4:-c3}
R=$(pwd)
for r in $(seq $rounds); do
  for arm in base new env; do
    if [ $arm = base ]; then dir=$R/$base; else dir=$R; fi
    if [ $arm = env ]; then ev="$envsw"; else ev="XTRL_AB_NOP=1"; fi
    (cd $dir && env "$ev" timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-loss-delta --no-roofline) > gpurun_out/abe_$arm.log 2>&1 || exit 1
    echo -n "$cfg $arm: "; tail -1 gpurun_out/abe_$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phase_ms'])"
  done
done
