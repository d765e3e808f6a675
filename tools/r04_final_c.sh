#!/bin/bash
# round-4 closing session C: a 2-rank rehearsal of the C5 gene-sharded DP path (gloo between two ranks
# sharing the one GPU) -> gpurun_out/final/ (progress on stderr, into the log)
set -u
mkdir -p gpurun_out/final
XTRL_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/final/r04_bench_2rank_gloo.log 2>&1
rc=$?; grep -h "bench rank\|Error\|error" gpurun_out/final/r04_bench_2rank_gloo.log | tail -12; tail -n 1 gpurun_out/final/r04_bench_2rank_gloo.log | cut -c1-400; exit $rc
