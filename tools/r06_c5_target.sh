set -u
mkdir -p gpurun_out
for r in 1 2; do
  for tg in 192 128 256; do
    XTRL_WGRAD_TARGET=$tg timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/c5t.log 2>&1 || exit 1
    echo -n "c5 target=$tg: "; tail -1 gpurun_out/c5t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
  done
done
