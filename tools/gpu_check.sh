#!/bin/bash
# One GPU session: parity tests, then (only if they did not crash the process) bench + profile.
# Usage: tools/gpu_check.sh [tests|bench|prof|all] [bench args...]
set -u
mkdir -p gpurun_out
what=${1:-all}; shift || true
run_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout=300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -15 gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
}
run_bench() {
  timeout -k 10 900 python bench.py "$@" > gpurun_out/bench.log 2>&1
  rc=$?; tail -5 gpurun_out/bench.log
  if [ $rc -ne 0 ]; then echo "bench rc=$rc: stopping"; exit $rc; fi
}
# output suffix of a non-default bench config (--config c5 -> _c5), matching bench.py _profile()
sfx() {
  local prev=""
  for a in "$@"; do
    if [ "$prev" = "--config" ] && [ "$a" != "c3" ]; then echo "_$a"; return; fi
    prev=$a
  done
}
run_prof() {
  local S=$(sfx "$@")
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof$S -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $GRAFT_REPO_ROOT/gpurun_out/prof$S.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; tail -3 gpurun_out/prof$S.log
  find gpurun_out/prof$S -type f ! -name '*stats*' -delete
  if [ $rc -ne 0 ]; then echo "prof rc=$rc"; exit $rc; fi
}
run_pmc() {
  # HBM traffic counters, one counter group per pass (FETCH_SIZE and WRITE_SIZE do not fit together)
  local S=$(sfx "$@")
  cd /tmp && export TMPDIR=/tmp
  # one counter group per pass: HBM read bytes, HBM write bytes, MFMA busy cycles + GPU clock
  for c in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    name=$(echo $c | cut -d' ' -f1)
    # only the two roofline kernels (many more dispatches crash the counter-collection tool)
    timeout -k 10 900 rocprofv3 --pmc $c --kernel-include-regex "k_attn_decode|k_gemm<2, 2, 1, 2, 2, true, true|k_gemm_ws<true, true" -d $GRAFT_REPO_ROOT/gpurun_out/pmc$S/pmc_$name -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-loss-delta "$@" > $GRAFT_REPO_ROOT/gpurun_out/pmc${S}_$name.log 2>&1
    rc=$?; tail -2 $GRAFT_REPO_ROOT/gpurun_out/pmc${S}_$name.log
    if [ $rc -ne 0 ]; then echo "pmc $c rc=$rc"; exit $rc; fi
  done
  cd $GRAFT_REPO_ROOT && python3 tools/pmc_summary.py gpurun_out/pmc$S > gpurun_out/pmc_summary$S.txt; cat gpurun_out/pmc_summary$S.txt
}
run_trace() {
  # kernel trace of one update (tools/update_trace.py): per-phase totals, one minibatch, one decode step
  local cfg=${1:-c3}
  local S=$(sfx --config $cfg)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/trace$S -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/update_trace.py run $cfg > $GRAFT_REPO_ROOT/gpurun_out/trace$S.log 2>&1
  rc=$?; cd $GRAFT_REPO_ROOT; tail -3 gpurun_out/trace$S.log
  if [ $rc -ne 0 ]; then echo "trace rc=$rc"; exit $rc; fi
  python3 tools/update_trace.py show $(find gpurun_out/trace$S -name '*kernel_trace.csv' | head -1) > gpurun_out/trace_summary$S.txt
  find gpurun_out/trace$S -type f -name '*kernel_trace.csv' -delete
  head -80 gpurun_out/trace_summary$S.txt
}
case $what in
  trace) run_trace "$@" ;;
  pmc) run_pmc "$@" ;;
  tests) run_tests ;;
  bench) run_bench "$@" ;;
  prof) run_prof "$@" ;;
  all) run_tests; run_bench "$@"; run_prof "$@" ;;
esac
