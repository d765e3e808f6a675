# row GEMV k-group cap A/B (ROW_KG_MAX 32 / 16 / 8 builds under tools/kg): phase stamps + lander_host
set -o pipefail
mkdir -p gpurun_out/kg
for kg in 32 16 8; do
  XTRL_LIB=kgbuild/libxtrl_kg$kg.so timeout -k 10 200 python tools/row_stamps.py > gpurun_out/kg/st$kg.txt 2>&1 || exit 1
  echo "== kg $kg"; grep "t=64\|stamping 0" gpurun_out/kg/st$kg.txt | cut -c1-200 | head -3
done
for r in 1 2; do for kg in 32 16 8; do
  XTRL_LIB=kgbuild/libxtrl_kg$kg.so timeout -k 10 200 python bench.py --config lander_host --steps 2 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/kg/b.log 2>&1 || exit 1
  echo -n "kg $kg: "; tail -1 gpurun_out/kg/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
done; done
