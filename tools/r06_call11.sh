#!/bin/bash
set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
  -k "c5 or fractal or gemm" > gpurun_out/r06_t11.log 2>&1
rc=$?; tail -3 gpurun_out/r06_t11.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
bash tools/ab_tree.sh abh 2 c5 || exit 1
bash tools/ab_tree.sh abh 1 c3 || exit 1
