#!/bin/bash
# stamp-free ws GEMM modes (tools/ws_lab.hip, -DXTRL_WS_MODE): full / no MFMA / no loads+splits / loads only /
# loads + LDS writes without the split arithmetic
set -u
mkdir -p gpurun_out; out=gpurun_out/wslab_modes.txt; : > $out
for m in 0 1 2 3 4; do
  hipcc -O3 -std=c++17 -fno-slp-vectorize --offload-arch=gfx950 -DXTRL_WS_MODE=$m -Ix-transformers-rl_amd/csrc tools/ws_lab.hip -o /tmp/wsm$m 2>/dev/null || exit 3
done
for shape in "1024 256 16384 1 1 0 1376" "1024 256 16384 1 1 0 1024" "256 1024 16384 1 1 0 1376" "16384 256 1024 0 1 0 0" "16384 1024 256 0 0 0 0"; do
  for m in 0 1 2 3 4; do
    timeout -k 10 60 /tmp/wsm$m $shape >> $out 2>&1 || { echo "fail rc=$?"; exit 1; }
  done
done
cat $out
