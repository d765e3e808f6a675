#!/bin/bash
# K keys per round trip in the row-resident step's attention (dh 16): 256 (default) vs 128, C2 bench
set -u
mkdir -p gpurun_out
bash tools/ab_env.sh XTRL_ROW_KP 4 2 3 c2
