# LayerNorm gains staged in LDS once per launch (gn build) vs read per LayerNorm phase: stamps + lander_host
set -o pipefail
mkdir -p gpurun_out/gn
for v in base gn; do
  XTRL_LIB=kgbuild/libxtrl_$v.so timeout -k 10 200 python tools/row_stamps.py > gpurun_out/gn/st_$v.txt 2>&1 || exit 1
  echo "== $v"; grep "t=64\|stamping 0" gpurun_out/gn/st_$v.txt | sed 's/.*\(lnf.*\)/\1/' | head -3
done
for r in 1 2; do for v in base gn; do
  XTRL_LIB=kgbuild/libxtrl_$v.so timeout -k 10 200 python bench.py --config lander_host --steps 2 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/gn/b.log 2>&1 || exit 1
  echo -n "$v: "; tail -1 gpurun_out/gn/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
done; done
