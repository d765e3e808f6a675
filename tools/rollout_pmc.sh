#!/bin/bash
# PMC counters of the rollout's small kernels (one counter group per pass).  Usage: tools/rollout_pmc.sh REGEX
set -u
mkdir -p gpurun_out
re=${1:-"k_embed|k_sample|k_compact"}
cd /tmp && export TMPDIR=/tmp
i=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
         "SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "$re" -d $GRAFT_REPO_ROOT/gpurun_out/pmc$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/rollout_probe.py --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc$i.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob('gpurun_out/pmc*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)', '').split('(')[0][-40:]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        n[(k, r['Counter_Name'])] += 1
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f'   {c:28s} {v / max(n[(k, c)], 1):14.1f} per dispatch')
PY
find gpurun_out/pmc* -name '*counter_collection.csv' -delete
