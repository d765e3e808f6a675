set -o pipefail
mkdir -p gpurun_out/row
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "rollout or row_step or host_env or learner_replays" > gpurun_out/row/t.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/row/t.log; exit 1; }
tail -2 gpurun_out/row/t.log
for arm in 1 0 1 0; do
  XTRL_ROW_SMALL=$arm timeout -k 10 200 python bench.py --config lander_host --steps 2 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/row/b$arm.log 2>&1 || exit 1
  echo -n "small=$arm: "; tail -1 gpurun_out/row/b$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'], d.get('host_step_us'))"
done
