#!/bin/bash
# C2 learn: per-launch grid and duration of the training attention kernels
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/attn_c2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for SPL in 1 2 4; do
XTRL_ATTN_SPLIT=$SPL timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "k_attn" -d $O/s$SPL -o run --output-format csv -- python3 $R/bench.py --config c2 --steps 1 --warmup 1 --no-cpu-baseline > $O/log$SPL.txt 2>&1 || exit $?
done
cd $R; find gpurun_out/attn_c2 -name "*.csv" ! -name "*kernel_trace*" -delete
