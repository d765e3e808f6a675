#!/bin/bash
# instruction-cache counters of the row-resident decode step (lander_host shape), one PMC pass each
cd /tmp && export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/ric
for pmc in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
  tag=$(echo $pmc | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex decode_row -d $out/$tag -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/row_stamps.py > $out.$tag.log 2>&1 || { echo "pmc pass $tag failed"; tail -5 $out.$tag.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob, collections
for f in glob.glob('gpurun_out/ric/*/**/*counter_collection.csv', recursive=True):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
    print(f.split('/')[2], {k: (len(v), sum(v) / len(v)) for k, v in acc.items()})
PY
