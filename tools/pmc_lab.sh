set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_lab
i=0
for c in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_lab/p$i -o run --output-format csv -- $R/tools/ws_lab.bin 16384 256 1024 > $R/gpurun_out/pmc_lab/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc_lab/p$i.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob('gpurun_out/pmc_lab/p*/**/*counter_collection.csv', recursive=True)):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        if 'k_gemm_ws' in row.get('Kernel_Name', ''):
            acc[row['Counter_Name']].append(float(row['Counter_Value']))
    for k, v in acc.items(): print(f.split('/')[2], k, 'per launch', sum(v) / max(1, len(set(range(len(v))))) if False else sum(v)/13)
PY
