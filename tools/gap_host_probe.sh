#!/bin/bash
# C5 / C3 learn idle gaps vs host launch times (kernel + HIP API trace, no counters)
cfg=${1:-c5}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/gaph_$cfg; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $O -o run --output-format csv -- python3 $R/bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline > $O/log.txt 2>&1
rc=$?; cd $R
[ $rc -eq 0 ] && python3 tools/gap_host_probe.py $O > $O/summary.txt 2>&1
find $O -name "*.csv" ! -name "*hip_api_trace.csv" -delete; python3 - <<EOP
import csv,glob
f=glob.glob("$O/**/*hip_api_trace.csv",recursive=True)
print(open(f[0]).readline() if f else "none")
EOP
find $O -name "*.csv" -delete; cat $O/summary.txt; exit $rc
