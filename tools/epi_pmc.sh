#!/bin/bash
# SQ counter passes over tools/epi_gemm_lab (build/epi_gemm_lab): where the FF1-shaped GEMM's waves
# spend their cycles with the plain / GELU / GELU + derivative (+ dropout) epilogues
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/epi_pmc
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SALU" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVES"; do
  name=$(echo $set | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex "k_gemm" -d $R/gpurun_out/epi_pmc/$name -o run --output-format csv -- $R/build/epi_gemm_lab > $R/gpurun_out/epi_pmc/$name.log 2>&1
  rc=$?
  echo "$set rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
cd $R && python3 - <<'PY'
import csv, glob
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob('gpurun_out/epi_pmc/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void xtrl::', '')
        acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in sorted(acc.items()):
    print(k, ' dispatches', len(d.get('SQ_WAVES', [])))
    for c, v in sorted(d.items()):
        print(f'   {c:28s} {sum(v) / len(v):14.0f}')
PY
find gpurun_out/epi_pmc -name '*.csv' -delete
