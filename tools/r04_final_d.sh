#!/bin/bash
# round-4 closing session D: C2 profiles at the default one workgroup per row; 2-rank gloo rehearsals
# (two ranks sharing the one GPU) of C3 and C5 -> gpurun_out/final/
set -u
mkdir -p gpurun_out/final
bash tools/final_profiles.sh r04 c2 || exit $?
for cfg in c3 c5; do
  XTRL_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-loss-delta > gpurun_out/final/r04_bench_2rank_gloo_$cfg.log 2>&1 || exit $?
  echo "$cfg: $(tail -n 1 gpurun_out/final/r04_bench_2rank_gloo_$cfg.log | cut -c1-300)"
done
