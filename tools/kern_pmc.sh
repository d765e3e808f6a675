#!/bin/bash
# SQ counter passes (one group per run) on the kernels matching $1 during one C3 bench step:
# where a kernel's waves spend their cycles (busy / waiting / VALU / LDS / memory instructions)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
re=$1
mkdir -p $R/gpurun_out/kern_pmc
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVES"; do
  name=$(echo $set | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "$re" -d $R/gpurun_out/kern_pmc/$name -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-loss-delta --no-roofline > $R/gpurun_out/kern_pmc/$name.log 2>&1
  rc=$?
  echo "$set rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
cd $R && python3 - <<'PY'
import csv, glob
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob('gpurun_out/kern_pmc/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void xtrl::', '')
        acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in sorted(acc.items()):
    print(k, ' dispatches', len(d.get('SQ_WAVES', [])))
    for c, v in sorted(d.items()):
        print(f'   {c:28s} {sum(v) / len(v):14.0f}')
PY
find gpurun_out/kern_pmc -name '*.csv' -delete
