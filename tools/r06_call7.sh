#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config c2_tok --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/b_c2tok.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/b_c2tok.log; exit 1; }
tail -1 gpurun_out/b_c2tok.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2_tok', d['value'], d['phase_ms'], d['ppo_loss'], d['roofline']['frac'])"
for v in 128 256; do
  XTRL_WGRAD_TARGET=$v timeout -k 10 300 python bench.py --config c2 --steps 4 --warmup 2 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/ab_t$v.log 2>&1 || exit 1
  echo -n "c2 target=$v: "; tail -1 gpurun_out/ab_t$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
done
timeout -k 10 300 python bench.py --config c2 --steps 4 --warmup 2 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/ab_t192.log 2>&1 || exit 1
echo -n "c2 target=192: "; tail -1 gpurun_out/ab_t192.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
XTRL_GEMM_WS=0 timeout -k 10 300 python bench.py --config c2 --steps 4 --warmup 2 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/ab_ws0.log 2>&1 || exit 1
echo -n "c2 ws=0: "; tail -1 gpurun_out/ab_ws0.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
