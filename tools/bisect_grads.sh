#!/bin/bash
# the gradient-parity case that moves with the row-resident step's workgroups per row
set -u
mkdir -p gpurun_out
T='tests/test_gpu_parity.py::test_ppo_loss_and_grads_identical_weights'
for env in "XTRL_ROW_G=4" "XTRL_ROW_G=2"; do
  env $env timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 240 --timeout-method thread "$T" > gpurun_out/bisect.log 2>&1
  echo "$env: $(tail -1 gpurun_out/bisect.log)"
  grep -h "AssertionError: (" gpurun_out/bisect.log | head -3 | cut -c1-1500
done
exit 0
