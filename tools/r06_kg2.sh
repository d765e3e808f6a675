# row GEMV k-group cap A/B, round 2: lander_host with cap 4 / 8, C2 rollout with 32 / 16 / 8 / 4
set -o pipefail
mkdir -p gpurun_out/kg
for kg in 8 4; do
  XTRL_LIB=kgbuild/libxtrl_kg$kg.so timeout -k 10 200 python tools/row_stamps.py > gpurun_out/kg/st$kg.txt 2>&1 || exit 1
  echo "== kg $kg"; grep "t=64\|stamping 0" gpurun_out/kg/st$kg.txt | cut -c1-200 | head -2
done
for kg in 32 16 8 4; do
  XTRL_LIB=kgbuild/libxtrl_kg$kg.so timeout -k 10 300 python bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/kg/c2.log 2>&1 || exit 1
  echo -n "c2 kg $kg: "; tail -1 gpurun_out/kg/c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
done
