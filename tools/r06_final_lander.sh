#!/bin/bash
# lander_host line after the gated scalar-env loop: kernel stats (rocprofv3) + the bench line with its CPU baseline
set -u
mkdir -p gpurun_out/final
bash tools/gpu_check.sh prof --config lander_host || exit $?
cp gpurun_out/prof_lander_host/run_kernel_stats.csv gpurun_out/final/r06_kernel_stats_lander_host.csv
timeout -k 10 900 python bench.py --config lander_host > gpurun_out/final/bench_lander_host.log 2>&1 || exit $?
tail -n 1 gpurun_out/final/bench_lander_host.log > gpurun_out/final/r06_bench_lander_host.json
python3 -c "import json; d=json.load(open('gpurun_out/final/r06_bench_lander_host.json')); print(d['value'], d['phase_ms'], d['cpu_baseline']['value'], {k: v for k, v in d['host_step_us'].items() if k != 'note'})"
