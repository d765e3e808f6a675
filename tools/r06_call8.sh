#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  -k "packed_learn or c3_bench_minibatch or fused_train_step or gemm" > gpurun_out/r06_t8.log 2>&1
rc=$?; tail -4 gpurun_out/r06_t8.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "Error|error|assert" gpurun_out/r06_t8.log | head -20; exit $rc; }
bash tools/ab_env.sh XTRL_LN_THIN 0 1 2 c3_tok || exit 1
