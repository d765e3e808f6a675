#!/bin/bash
# standalone wgrad GEMM (FF1 shape of C3): kernel time vs split target + L2 / HBM counters
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/wgp; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for tgt in 192 96 128 256; do
  XTRL_WGRAD_TARGET=$tgt timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/t$tgt -o run --output-format csv -- python3 $R/tools/gemm_one.py wgrad 1024 256 16384 > $O/t$tgt.log 2>&1 || exit $?
done
for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum"; do
  name=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "k_gemm" -d $O/$name -o run --output-format csv -- python3 $R/tools/gemm_one.py wgrad 1024 256 16384 > $O/$name.log 2>&1 || exit $?
done
cd $R; find gpurun_out/wgp -type f -name '*kernel_stats*' -o -type f -name '*counter_collection*' | sort
