# the fractal backward's input-projection gradient on the main stream (XTRL_WPIN_MAIN): fractal learn parity, C5 learn A/B
set -o pipefail
mkdir -p gpurun_out/wpin
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "fractal" > gpurun_out/wpin/t5.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/wpin/t5.log; exit 1; }
tail -1 gpurun_out/wpin/t5.log
for r in 1 2; do for v in 0 1; do
  XTRL_WPIN_MAIN=$v timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/wpin/c5.log 2>&1 || exit 1
  echo -n "c5 wpin_main=$v: "; tail -1 gpurun_out/wpin/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
done; done
