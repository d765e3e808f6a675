#!/bin/bash
# Round-end measurement of one bench config on the GPU box: rocprofv3 kernel stats and the PMC
# passes (tools/gpu_check.sh), their summaries installed as profiles/rNN_*[_cfg] so the bench line
# quotes them, then the bench itself (with the CPU baseline).  Everything kept lands in
# gpurun_out/final/ (copied into profiles/ by hand afterwards).
# Usage: tools/final_profiles.sh <round tag, e.g. r03> <config: c3 | c2 | c5>
set -u
tag=$1; cfg=$2
S=""; [ "$cfg" != "c3" ] && S="_$cfg"
mkdir -p gpurun_out/final
bash tools/gpu_check.sh prof --config $cfg || exit $?
cp gpurun_out/prof$S/run_kernel_stats.csv profiles/${tag}_kernel_stats$S.csv
cp gpurun_out/prof$S/run_kernel_stats.csv gpurun_out/final/${tag}_kernel_stats$S.csv
bash tools/gpu_check.sh pmc --config $cfg || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc$S > profiles/${tag}_pmc_traffic$S.json
cp profiles/${tag}_pmc_traffic$S.json gpurun_out/final/
timeout -k 10 900 python bench.py --config $cfg > gpurun_out/final/bench$S.log 2>&1
rc=$?
tail -n 1 gpurun_out/final/bench$S.log > gpurun_out/final/${tag}_bench$S.json
exit $rc
