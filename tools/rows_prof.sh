#!/bin/bash
# kernel stats of the C2 bench (multi-kernel + row-resident decode steps) and the host-step probe
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_rows -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-loss-delta > $GRAFT_REPO_ROOT/gpurun_out/prof_rows.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $GRAFT_REPO_ROOT
find gpurun_out/prof_rows -type f ! -name '*kernel_stats*' -delete
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_rows/**/*kernel_stats.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:90]}")
PY
timeout -k 10 300 python tools/host_step_probe.py 2>&1 | grep -v amdgpu.ids
