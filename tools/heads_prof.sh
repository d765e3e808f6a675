#!/bin/bash
# kernel stats of the C3 bench with the one-launch heads (XTRL_DECODE_HEADS=1) vs the two-launch pair
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  XTRL_DECODE_HEADS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_heads$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-loss-delta > $GRAFT_REPO_ROOT/gpurun_out/prof_heads$v.log 2>&1 || { echo "prof rc=$?"; exit 1; }
done
cd $GRAFT_REPO_ROOT
find gpurun_out/prof_heads0 gpurun_out/prof_heads1 -type f ! -name '*kernel_stats*' -delete
python3 - <<'PY'
import csv, glob
for v in '10':
    f = glob.glob(f'gpurun_out/prof_heads{v}/**/*kernel_stats.csv', recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))
    print('XTRL_DECODE_HEADS', v)
    for r in rows:
        n = r['Name']
        if any(k in n for k in ('heads', 'k_dgemm', 'k_mlp', 'k_attn_decode', 'k_embed<')):
            print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.1f} us  {n[:90]}")
PY
