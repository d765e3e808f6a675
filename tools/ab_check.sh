#!/bin/bash
# A/B of a library env switch: parity tests, then the C3 bench with the switch at each value.
# Usage: tools/ab_check.sh VAR "v1 v2 ..."
set -u
mkdir -p gpurun_out
var=$1; vals=$2
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
for v in $vals; do
  env $var=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo "$var=$v"; tail -1 gpurun_out/ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phase_ms'])"
done
