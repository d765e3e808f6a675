#!/bin/bash
# row-resident step with / without the GEMV weight prefetch across the LayerNorm phases: parity of
# the row path, then C2 A/B against the saved base build and the host-step probe
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "rows or c2_full_width or host_env" > gpurun_out/rowpre_tests.log 2>&1
rc=$?; tail -2 gpurun_out/rowpre_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_lib.sh abx/libxtrl_base.so 3 c2 || exit 1
for lib in abx/libxtrl_base.so x-transformers-rl_amd/xtrl_amd/libxtrl_hip.so; do
  echo "host probe $lib"; XTRL_LIB=$lib timeout -k 10 120 python tools/host_step_probe.py 2>&1 | grep "decode step"
done
