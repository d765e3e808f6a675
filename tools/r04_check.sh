#!/bin/bash
# round-4 GPU session: the fused attention backward's kernel in a profile of its parity test, the
# whole -m gpu suite, then the C3 bench.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fused -o run --output-format csv -- python3 -m pytest -x -q -p no:cacheprovider $GRAFT_REPO_ROOT/tests/test_gpu_parity.py -k fused_backward_matches > $GRAFT_REPO_ROOT/gpurun_out/prof_fused.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $GRAFT_REPO_ROOT
grep -h "k_attn_bwd" $(find gpurun_out/prof_fused -name '*kernel_stats.csv') | cut -c1-120
find gpurun_out/prof_fused -type f ! -name '*stats*' -delete
bash tools/gpu_check.sh tests || exit $?
bash tools/gpu_check.sh bench --steps 10 --warmup 3 --no-cpu-baseline || exit $?
timeout -k 10 300 python bench.py --config lander_host --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_lander_host.log 2>&1 || { echo "lander_host rc=$?"; tail -20 gpurun_out/bench_lander_host.log; exit 1; }
tail -1 gpurun_out/bench_lander_host.log | cut -c1-400
