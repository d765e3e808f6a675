#!/bin/bash
set -u
bash tools/final_profiles.sh r06 c2 || exit $?
bash tools/final_profiles.sh r06 c5 || exit $?
for c in c2 c5; do cat gpurun_out/final/r06_bench_$c.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['phase_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"; done
