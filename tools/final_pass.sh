set -u
mkdir -p gpurun_out
bash tools/gpu_check.sh prof && bash tools/gpu_check.sh pmc > gpurun_out/pmc_run.log 2>&1 && bash tools/gpu_check.sh trace > /dev/null && \
timeout -k 10 600 python bench.py > gpurun_out/bench_c3.log 2>&1 && tail -1 gpurun_out/bench_c3.log && \
timeout -k 10 600 python bench.py --config c2 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 && tail -1 gpurun_out/bench_c2.log | cut -c1-300 && \
timeout -k 10 600 python bench.py --config c5 > gpurun_out/bench_c5.log 2>&1 && tail -1 gpurun_out/bench_c5.log | cut -c1-300
