# host-env / rollout parity after the per-wave host trims, then lander_host x2
set -o pipefail
mkdir -p gpurun_out/gate
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "host_env or rollout or row_step or learner_replays or c2_full or c3_full" > gpurun_out/gate/t3.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/gate/t3.log; exit 1; }
tail -2 gpurun_out/gate/t3.log
for arm in 1 1; do
  timeout -k 10 200 python bench.py --config lander_host --steps 2 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/gate/bb.log 2>&1 || { tail -20 gpurun_out/gate/bb.log; exit 1; }
  tail -1 gpurun_out/gate/bb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'], {k: v for k, v in d.get('host_step_us', {}).items() if k != 'note'})"
done
