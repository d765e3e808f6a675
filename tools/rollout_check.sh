mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "dgemm or rollout or deploy or host_env or e2e" > gpurun_out/t1.log 2>&1
rc=$?; tail -3 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/rp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/rollout_probe.py --reps 2 > $GRAFT_REPO_ROOT/gpurun_out/rp.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT; find gpurun_out/rp -type f ! -name "*stats*" -delete
timeout -k 10 100 python3 tools/rollout_probe.py
