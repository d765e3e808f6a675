#!/bin/bash
# C5 round-end line on the final code (kernel stats, PMC, bench with its CPU baseline)
set -u
bash tools/final_profiles.sh r06 c5 || exit $?
cat gpurun_out/final/r06_bench_c5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['value'], d['value_median'], d['phase_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
