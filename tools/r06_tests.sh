#!/bin/bash
# the whole -m gpu suite, as the driver runs it at round end
set -u
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_gpu_tests.txt 2>&1
rc=$?; tail -6 gpurun_out/r06_gpu_tests.txt; exit $rc
