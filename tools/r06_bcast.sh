# cross-row reductions on DPP row broadcasts (XTRL_DPP_BCAST): the GPU suite, stamps, lander_host / C3 rollout A/B vs the base build
set -o pipefail
mkdir -p gpurun_out/bc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/bc/t.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/bc/t.log; exit 1; }
tail -1 gpurun_out/bc/t.log
for v in base new; do
  if [ $v = base ]; then L=kgbuild/libxtrl_base.so; else L=x-transformers-rl_amd/xtrl_amd/libxtrl_hip.so; fi
  XTRL_LIB=$L timeout -k 10 200 python tools/row_stamps.py > gpurun_out/bc/st_$v.txt 2>&1 || exit 1
  echo "== $v"; grep "stamping 0" gpurun_out/bc/st_$v.txt | head -1
done
for r in 1 2; do for v in base new; do
  if [ $v = base ]; then L=kgbuild/libxtrl_base.so; else L=x-transformers-rl_amd/xtrl_amd/libxtrl_hip.so; fi
  XTRL_LIB=$L timeout -k 10 200 python bench.py --config lander_host --steps 2 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/bc/b.log 2>&1 || exit 1
  echo -n "lander_host $v: "; tail -1 gpurun_out/bc/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
  XTRL_LIB=$L timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/bc/c3.log 2>&1 || exit 1
  echo -n "c3 $v: "; tail -1 gpurun_out/bc/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
done; done
