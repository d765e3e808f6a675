#!/bin/bash
# rocprofv3 kernel trace of one C3 update (or $2), summarised by tools/update_trace.py into gpurun_out/${1:-r05_update_trace}.txt
name=${1:-r05_update_trace}; cfg=${2:-c3}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/update_trace.py run $cfg > $GRAFT_REPO_ROOT/gpurun_out/tr.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/tr -name '*kernel_trace.csv' | head -1)
python3 tools/update_trace.py show $f > gpurun_out/$name.txt 2>&1
rm -rf gpurun_out/tr
