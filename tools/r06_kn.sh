# the row step's new-key score as a DPP row sum (DH 16) vs 32 lane permutes: parity, stamps, lander_host A/B vs the base build
set -o pipefail
mkdir -p gpurun_out/kn
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "host_env or rollout or row_step or learner_replays or c2_full" > gpurun_out/kn/t.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/kn/t.log; exit 1; }
tail -1 gpurun_out/kn/t.log
for v in base new; do
  if [ $v = base ]; then L=kgbuild/libxtrl_base.so; else L=x-transformers-rl_amd/xtrl_amd/libxtrl_hip.so; fi
  XTRL_LIB=$L timeout -k 10 200 python tools/row_stamps.py > gpurun_out/kn/st_$v.txt 2>&1 || exit 1
  echo "== $v"; grep "t=64" gpurun_out/kn/st_$v.txt | cut -c1-90; grep "stamping 0" gpurun_out/kn/st_$v.txt | head -1
done
for r in 1 2; do for v in base new; do
  if [ $v = base ]; then L=kgbuild/libxtrl_base.so; else L=x-transformers-rl_amd/xtrl_amd/libxtrl_hip.so; fi
  XTRL_LIB=$L timeout -k 10 200 python bench.py --config lander_host --steps 2 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/kn/b.log 2>&1 || exit 1
  echo -n "lander_host $v: "; tail -1 gpurun_out/kn/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
done; done
