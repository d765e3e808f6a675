#!/bin/bash
# round-6 first GPU call: the new multi-GPU / compact-heads / alive tests, the ws-GEMM modes, the attention sweep
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_parity.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  -k "world1_rccl or self_launches or compact_world_model or oversubscribed" > gpurun_out/r06_t1.log 2>&1
rc=$?; tail -15 gpurun_out/r06_t1.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
bash tools/wslab_modes.sh > /dev/null 2>&1; rc=$?; cat gpurun_out/wslab_modes.txt
[ $rc -eq 0 ] || { echo "wslab rc=$rc"; exit $rc; }
bash tools/attn_sweep.sh
