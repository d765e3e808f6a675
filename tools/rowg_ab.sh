#!/bin/bash
# workgroups per row of the row-resident step: C2 bench and the host-step probe at 1 and 4
set -u
mkdir -p gpurun_out
bash tools/ab_env.sh XTRL_ROW_G 1 4 2 c2 || exit 1
for g in 1 4; do
  echo "host probe XTRL_ROW_G=$g"
  XTRL_ROW_G=$g timeout -k 10 120 python tools/host_step_probe.py 2>&1 | grep -v amdgpu.ids
done
