#!/bin/bash
# A/B of environment switches on one box: bench.py (C3, no CPU baseline / loss check) per setting,
# one JSON line each into gpurun_out/ab_<tag>.log.  Usage: tools/ab_env_bench.sh "tag:VAR=v VAR2=w" ...
mkdir -p gpurun_out
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-loss-delta > gpurun_out/ab_$tag.log 2>&1
  rc=$?
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1]);print('$tag', d['value'], d['phase_ms'], d['roofline']['frac'] if d.get('roofline') else None)" || echo "$tag failed rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
