#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  -k "packed_learn" > gpurun_out/r06_t9.log 2>&1
rc=$?; tail -12 gpurun_out/r06_t9.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "Error|error|assert" gpurun_out/r06_t9.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py --config c3_tok > gpurun_out/b_c3tok_final.log 2>&1 || { echo "bench rc=$?"; tail -3 gpurun_out/b_c3tok_final.log; exit 1; }
tail -1 gpurun_out/b_c3tok_final.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3_tok', d['value'], d['phase_ms'], d['roofline'])"
