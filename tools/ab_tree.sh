#!/bin/bash
# A/B of this tree against a saved worktree of an earlier commit (its own Python + in-tree library,
# e.g. `git worktree add abr05 <commit>` + make): bench.py alternating base / new, N rounds.
# Usage: tools/ab_tree.sh <base dir> [rounds] [config]
set -u
mkdir -p gpurun_out
base=$1; rounds=${2:-2}; cfg=${3:-c3}
R=$(pwd)
for r in $(seq $rounds); do
  for arm in base new; do
    if [ $arm = base ]; then dir=$R/$base; else dir=$R; fi
    (cd $dir && timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-loss-delta --no-roofline) > gpurun_out/abt_$arm.log 2>&1 || exit 1
    echo -n "$cfg $arm: "; tail -1 gpurun_out/abt_$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phase_ms'])"
  done
done
