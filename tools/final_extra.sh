#!/bin/bash
# Round-end lines of the extra bench configs (no PMC passes): rocprofv3 kernel stats of a short run,
# then the bench itself with its CPU baseline.  Usage: tools/final_extra.sh <round tag> <config>...
set -u
tag=$1; shift
mkdir -p gpurun_out/final
for cfg in "$@"; do
  bash tools/gpu_check.sh prof --config $cfg > gpurun_out/final/prof_$cfg.txt 2>&1 || { echo "prof $cfg failed"; exit 1; }
  cp gpurun_out/prof_$cfg/run_kernel_stats.csv gpurun_out/final/${tag}_kernel_stats_$cfg.csv
  timeout -k 10 900 python bench.py --config $cfg > gpurun_out/final/bench_$cfg.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/final/bench_$cfg.log; exit 1; }
  tail -n 1 gpurun_out/final/bench_$cfg.log > gpurun_out/final/${tag}_bench_$cfg.json
  echo "$cfg done"
done
