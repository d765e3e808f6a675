#!/bin/bash
# distributed GPU tests, then the 2-rank gloo rehearsals (C3, C5) -> gpurun_out/final/
set -u
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -p no:cacheprovider tests/test_gpu_distributed.py > gpurun_out/final/dist_tests.log 2>&1
rc=$?; tail -2 gpurun_out/final/dist_tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in c3 c5; do
  XTRL_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-loss-delta > gpurun_out/final/r04_bench_2rank_gloo_$cfg.log 2>&1 || exit $?
  echo "$cfg: $(tail -n 1 gpurun_out/final/r04_bench_2rank_gloo_$cfg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["phase_ms"], d.get("dp"))')"
done
