#!/bin/bash
# split-K target of the weight-gradient GEMMs (workgroups of a 128 x 128-tile launch), C3 learn
set -u
mkdir -p gpurun_out
bash tools/ab_env.sh XTRL_WGRAD_TARGET 192 256 2 c3 || exit 1
bash tools/ab_env.sh XTRL_WGRAD_TARGET 192 144 2 c3
