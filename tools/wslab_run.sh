set -u
mkdir -p gpurun_out
B=/tmp/ws_lab.bin
hipcc -O3 -std=c++17 -fno-slp-vectorize --offload-arch=gfx950 -DXTRL_WS_DIAG -Ix-transformers-rl_amd/csrc tools/ws_lab.hip -o $B 2>/dev/null || exit 3
for shape in "1024 256 16384 1 1 MODE 1376" "256 1024 16384 1 1 MODE 1376" "768 256 16384 1 1 MODE 2752"; do
  for m in 0 1 2 3; do
    args=${shape/MODE/$m}
    timeout -k 10 60 $B $args >> gpurun_out/wslab.txt 2>&1 || { echo "fail rc=$?"; exit 1; }
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES -d $GRAFT_REPO_ROOT/gpurun_out/wspmc -o run --output-format csv -- $B 1024 256 16384 1 1 0 1376 > $GRAFT_REPO_ROOT/gpurun_out/wspmc.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; cat gpurun_out/wslab.txt; exit $rc
