#!/bin/bash
# k_attn_decode sweep (tools/attn_sweep.py): HIP events, then a rocprofv3 kernel trace and the two
# HBM-counter passes of the same sweep, summarised per (t, live rows) point.
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 tools/attn_sweep.py run --out $R/gpurun_out/attn_sweep.json > gpurun_out/attn_sweep.log 2>&1 || { echo "sweep rc=$?"; tail -20 gpurun_out/attn_sweep.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/asw_trace -o run --output-format csv -- python3 $R/tools/attn_sweep.py run --out $R/gpurun_out/attn_sweep_t.json > $R/gpurun_out/asw_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "k_attn_decode" -d $R/gpurun_out/asw_$c -o run --output-format csv -- python3 $R/tools/attn_sweep.py run --out $R/gpurun_out/attn_sweep_$c.json > $R/gpurun_out/asw_$c.log 2>&1 || { echo "pmc $c rc=$?"; exit 1; }
done
cd $R
python3 tools/attn_sweep.py summarize gpurun_out/attn_sweep.json gpurun_out/asw_trace gpurun_out/asw_FETCH_SIZE gpurun_out/asw_WRITE_SIZE > gpurun_out/attn_sweep_summary.txt 2>&1
cat gpurun_out/attn_sweep_summary.txt
find gpurun_out/asw_trace gpurun_out/asw_FETCH_SIZE gpurun_out/asw_WRITE_SIZE -type f -name '*.csv' ! -name '*kernel_trace*' ! -name '*counter_collection*' -delete 2>/dev/null
true
