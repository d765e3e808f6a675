set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or fused_train or ppo_loss" -p no:cacheprovider > gpurun_out/t_gemm.log 2>&1; rc=$?; tail -3 gpurun_out/t_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/gb_ws.log 2>&1 || exit $?
XTRL_GEMM_WS=0 timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/gb_old.log 2>&1 || exit $?
paste -d'\n' gpurun_out/gb_ws.log gpurun_out/gb_old.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ws.log 2>&1 || exit $?
tail -1 gpurun_out/bench_ws.log | cut -c1-400
