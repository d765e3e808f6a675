cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/update_trace.py run c3 > $GRAFT_REPO_ROOT/gpurun_out/tr.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/tr -name '*kernel_trace.csv' | head -1)
python3 tools/update_trace.py show $f > gpurun_out/r05_update_trace.txt 2>&1
rm -rf gpurun_out/tr
