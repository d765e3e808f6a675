#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  -k "packed_learn or attention_long or attention_fused or compact_world" > gpurun_out/r06_t5.log 2>&1
rc=$?; tail -15 gpurun_out/r06_t5.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "Error|error|assert" gpurun_out/r06_t5.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --config c3_tok --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_c3tok.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/b_c3tok.log; exit 1; }
tail -1 gpurun_out/b_c3tok.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3_tok', d['value'], d['phase_ms'], d['ppo_loss'], d['roofline']['frac'])"
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_c3.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/b_c3.log; exit 1; }
tail -1 gpurun_out/b_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['phase_ms'], d['ppo_loss'], d['roofline']['frac'])"
