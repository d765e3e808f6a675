# project_in's weight gradient on the main stream with the split-K flush started beside the embedding backward
# (XTRL_WPIN_MAIN=1, default) vs on the side stream before the flush: learn parity, then C3 / C2 learn A/B
set -o pipefail
mkdir -p gpurun_out/wpin
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "learn or grad or packed or compact or optimizer or ppo or c3_bench or c2_bench or c5_bench" > gpurun_out/wpin/t.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/wpin/t.log; exit 1; }
tail -1 gpurun_out/wpin/t.log
for r in 1 2; do for v in 0 1; do
  XTRL_WPIN_MAIN=$v timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/wpin/c3.log 2>&1 || exit 1
  echo -n "c3 wpin_main=$v: "; tail -1 gpurun_out/wpin/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
done; done
for v in 0 1; do
  XTRL_WPIN_MAIN=$v timeout -k 10 300 python bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/wpin/c2.log 2>&1 || exit 1
  echo -n "c2 wpin_main=$v: "; tail -1 gpurun_out/wpin/c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
done
