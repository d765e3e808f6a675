#!/bin/bash
# counter passes on the training attention kernels (tools/attn_bench.py), one counter group per run
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/attn_pmc
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD"; do
  name=$(echo $set | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex "k_attn" -d $R/gpurun_out/attn_pmc/$name -o run --output-format csv -- python3 $R/tools/attn_bench.py > $R/gpurun_out/attn_pmc/$name.log 2>&1
  rc=$?
  echo "$set rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
cd $R && python3 - <<'PY'
import csv, glob
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob('gpurun_out/attn_pmc/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void xtrl::', '')
        acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f'   {c:28s} {sum(v) / len(v):14.0f}')
PY
find gpurun_out/attn_pmc -name '*.csv' -delete
