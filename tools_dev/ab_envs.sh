#!/bin/bash
# A/B of environment settings on one box: bench (f32 B=1 + the bf16 batch extras + Q8 B=1)
# under each setting, alternating, N rounds. A setting is "-" (none) or VAR=VAL[,VAR=VAL].
# usage: tools_dev/ab_envs.sh TAG N SETTING [SETTING ...]
set -e -o pipefail
TAG=$1; N=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  k=0
  for S in "$@"; do
    k=$((k+1))
    (
      if [ "$S" != "-" ]; then for kv in ${S//,/ }; do export "$kv"; done; fi
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-codec --steps 10 > gpurun_out/${TAG}_${k}_${i}.log 2>&1
    )
    tail -1 gpurun_out/${TAG}_${k}_${i}.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d.get('extra_configs',{})
print('$S', round(d['value'],1), e.get('bf16_batch1_fps'), e.get('bf16_batch8_fps'), e.get('bf16_batch16_fps'), e.get('q8_batch1_fps'))"
  done
done
