#!/bin/bash
# kernel stats of the drop-in lander_host bench (scalar host env, row-resident decode step)
set -u
mkdir -p gpurun_out/final
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_lh -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config lander_host --steps 1 --warmup 1 --no-cpu-baseline --no-loss-delta > $GRAFT_REPO_ROOT/gpurun_out/prof_lh.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/prof_lh -name '*kernel_stats.csv' | head -1)
cp $f gpurun_out/final/r04_kernel_stats_lander_host.csv
find gpurun_out/prof_lh -type f ! -name '*kernel_stats*' -delete
python3 - <<'PY'
import csv
rows = sorted(csv.DictReader(open('gpurun_out/final/r04_kernel_stats_lander_host.csv')), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:10]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:80]}")
PY
