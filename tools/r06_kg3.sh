# ROW_KG_MAX 8 default: row / rollout / host-env parity, then the lander_host round-end line
set -o pipefail
mkdir -p gpurun_out/kg
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "host_env or rollout or row_step or learner_replays or c2_full" > gpurun_out/kg/t.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/kg/t.log; exit 1; }
tail -1 gpurun_out/kg/t.log
bash tools/r06_final_lander.sh
