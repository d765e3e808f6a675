#!/bin/bash
# A/B of an environment switch on one box: alternate VAR=a / VAR=b, N rounds [config]
set -u
var=$1; a=$2; b=$3; rounds=${4:-2}; cfg=${5:-c3}
for r in $(seq $rounds); do
  for v in $a $b; do
    env $var=$v timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-loss-delta --no-roofline > gpurun_out/ab_$v.log 2>&1 || exit 1
    echo -n "$cfg $var=$v: "; tail -1 gpurun_out/ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phase_ms'])"
  done
done
