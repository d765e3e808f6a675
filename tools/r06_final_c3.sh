#!/bin/bash
# round-6 final profile + bench of the headline config, then the update traces of c3 and c3_tok
set -u
bash tools/final_profiles.sh r06 c3 || exit $?
cat gpurun_out/final/r06_bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['phase_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
bash tools/gpu_check.sh trace c3 > /dev/null 2>&1 || exit 1
cp gpurun_out/trace_summary.txt gpurun_out/final/r06_update_trace.txt
bash tools/gpu_check.sh trace c3_tok > /dev/null 2>&1 || exit 1
cp gpurun_out/trace_summary_c3_tok.txt gpurun_out/final/r06_update_trace_c3_tok.txt
head -3 gpurun_out/final/r06_update_trace_c3_tok.txt
