# sampling inputs loaded at the row's start (ROW_SAMPLE_EARLY build) vs at the sampling: stamps + lander_host
set -o pipefail
mkdir -p gpurun_out/se
for v in base se; do
  XTRL_LIB=kgbuild/libxtrl_$v.so timeout -k 10 200 python tools/row_stamps.py > gpurun_out/se/st_$v.txt 2>&1 || exit 1
  echo "== $v"; grep "t=64\|stamping 0" gpurun_out/se/st_$v.txt | sed 's/.*\(lnf.*\)/\1/' | head -3
done
for r in 1 2; do for v in base se; do
  XTRL_LIB=kgbuild/libxtrl_$v.so timeout -k 10 200 python bench.py --config lander_host --steps 2 --warmup 1 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/se/b.log 2>&1 || exit 1
  echo -n "$v: "; tail -1 gpurun_out/se/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms'])"
done; done
