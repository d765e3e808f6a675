#!/bin/bash
# the row-resident decode step: its parity tests (both decode paths), then C2 / lander_host benches
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "rollout_matches_oracle or continuous_matches or graph_replay_equals or host_env or c2_full_width or smoke" > gpurun_out/rows_tests.log 2>&1
rc=$?; tail -15 gpurun_out/rows_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_c2.log 2>&1 || exit $?
tail -1 gpurun_out/b_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['phase_ms'])"
timeout -k 10 300 python bench.py --config lander_host --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_lh.log 2>&1 || exit $?
tail -1 gpurun_out/b_lh.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lander_host', d['value'], d['phase_ms'])"
