#!/bin/bash
set -u
mkdir -p gpurun_out
hipcc -O3 -std=c++17 -fno-slp-vectorize --offload-arch=gfx950 -Ix-transformers-rl_amd/csrc tools/wgrad_span_lab.hip -o /tmp/wsl 2>/dev/null || exit 3
timeout -k 10 120 /tmp/wsl > gpurun_out/wgrad_span_lab.txt 2>&1; rc=$?; cat gpurun_out/wgrad_span_lab.txt; exit $rc
