#!/bin/bash
set -u
mkdir -p gpurun_out
hipcc -O3 -std=c++17 -fno-slp-vectorize --offload-arch=gfx950 -Ix-transformers-rl_amd/csrc tools/cs_lab.hip -o /tmp/cs_lab 2>/dev/null || exit 3
timeout -k 10 120 /tmp/cs_lab > gpurun_out/cs_lab.txt 2>&1; rc=$?; cat gpurun_out/cs_lab.txt; exit $rc
