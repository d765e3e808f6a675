#!/bin/bash
# round-4 rollout changes: parity of the decode paths, then A/B of the fp32 vs split feed-forward
# images (C3) and of the row-resident step's workgroups per row (C2)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "ff_glu or fused_train_step_large or rollout_matches_oracle or continuous_matches or graph_replay_equals or host_env or full_width or smoke or fractal_decode or fractal_rollout" > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh XTRL_MLP_IMG x6 f32 2 c3 || exit 1
bash tools/ab_env.sh XTRL_MLP_EW 0 1 2 c3 || exit 1
bash tools/ab_env.sh XTRL_ROW_G 1 4 2 c2 || exit 1
bash tools/ab_env.sh XTRL_MLP_IMG x6 f32 1 c5 || exit 1
timeout -k 10 120 python tools/host_step_probe.py 2>&1 | grep -v amdgpu.ids
