#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  -k "attention_long_backward or attention_fused_backward or c2_bench_minibatch or c2_shape" > gpurun_out/r06_t2.log 2>&1
rc=$?; tail -15 gpurun_out/r06_t2.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
bash tools/ab_env.sh XTRL_ATTN_FUSED_BWD 0 1 2 c2 || exit 1
bash tools/wslab_modes.sh > /dev/null 2>&1; rc=$?; grep -E "^mode" gpurun_out/wslab_modes.txt
bash tools/gpu_check.sh trace c3 > /dev/null 2>&1; rc=$?; grep -A32 "by launch shape" gpurun_out/trace_summary.txt
exit $rc
