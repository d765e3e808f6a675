#!/bin/bash
# round-4 closing session A: the whole -m gpu suite, then the C3 profiles (rocprof kernel stats, PMC
# passes) and the C3 bench line with the CPU baseline (tools/final_profiles.sh) -> gpurun_out/final/
set -u
mkdir -p gpurun_out/final
bash tools/gpu_check.sh tests || exit $?
cp gpurun_out/gpu_tests.log gpurun_out/final/r04_gpu_tests.txt
bash tools/final_profiles.sh r04 c3
