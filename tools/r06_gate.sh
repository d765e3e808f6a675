# gated scalar-env loop: host-env parity tests, then lander_host A/B (gated vs launch-per-step)
set -o pipefail
mkdir -p gpurun_out/gate
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "host_env" > gpurun_out/gate/t.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/gate/t.log; exit 1; }
tail -2 gpurun_out/gate/t.log
for arm in 1 0 1 0; do
  XTRL_HOST_GATE=$arm timeout -k 10 200 python bench.py --config lander_host --steps 2 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/gate/b$arm.log 2>&1 || { tail -20 gpurun_out/gate/b$arm.log; exit 1; }
  echo -n "gate=$arm: "; tail -1 gpurun_out/gate/b$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'], {k: v for k, v in d.get('host_step_us', {}).items() if k != 'note'})"
done
