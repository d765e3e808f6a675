#!/bin/bash
# round-4 closing session B: C2 and C5 profiles + bench lines (tools/final_profiles.sh) -> gpurun_out/final/
set -u
mkdir -p gpurun_out/final
bash tools/final_profiles.sh r04 c2 || exit $?
bash tools/final_profiles.sh r04 c5
