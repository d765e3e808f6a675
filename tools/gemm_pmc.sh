#!/bin/bash
# counter passes on one GEMM shape: tools/gemm_pmc.sh <tag> <gemm_one.py args...>
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"; do
  name=$(echo $set | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex "k_gemm" -d $R/gpurun_out/pmc_$tag/$name -o run --output-format csv -- python3 $R/tools/gemm_one.py "$@" > $R/gpurun_out/pmc_$tag/$name.log 2>&1
  rc=$?
  echo "$set rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
exit 0
