#!/bin/bash
# Alternating A/B of environment settings on one box, f32 batch 1 headline only (plus the
# line's op table): tools_dev/ab_kv.sh TAG N "A=1" "A=0 B=2" ...   (each arg: space-separated K=V)
set -e -o pipefail
TAG=$1; N=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  j=0
  for kv in "$@"; do
    j=$((j + 1))
    env $kv timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-codec --no-extra --steps 20 \
      > gpurun_out/${TAG}_${j}_${i}.log 2>&1
    tail -1 gpurun_out/${TAG}_${j}_${i}.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); o=d.get('ops',{})
lt=sum(v['us_per_frame'] for k,v in o.items() if k.startswith('lt_') or k=='finalize')
print('[$kv]', round(d['value'],1), 'scale_b8', d['scaling_baseline']['value'], 'LT us/frame', round(lt,1),
      {k: v['avg_us'] for k,v in o.items() if k.startswith('lt_')})"
  done
done
