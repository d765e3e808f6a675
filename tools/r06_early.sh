# deferred split-K sums flushed before the first block's weight gradients (XTRL_SPLITK_EARLY=1) vs at the end: C3 / C5 learn A/B
set -o pipefail
mkdir -p gpurun_out/early
for r in 1 2; do for v in 0 1; do
  XTRL_SPLITK_EARLY=$v timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/early/c3.log 2>&1 || exit 1
  echo -n "c3 early=$v: "; tail -1 gpurun_out/early/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
done; done
for v in 0 1; do
  XTRL_SPLITK_EARLY=$v timeout -k 10 300 python bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/early/c2.log 2>&1 || exit 1
  echo -n "c2 early=$v: "; tail -1 gpurun_out/early/c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
done
