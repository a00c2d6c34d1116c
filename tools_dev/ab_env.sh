#!/bin/bash
# A/B of an environment switch on one box: bench (f32 B=1 + extras) with and without
# it, alternating, N rounds. Usage: tools_dev/ab_env.sh TAG VAR [N]
set -e -o pipefail
TAG=$1; VAR=$2; N=${3:-2}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for on in 0 1; do
    if [ $on = 1 ]; then export $VAR=1; else unset $VAR; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/${TAG}_${on}_${i}.log 2>&1
    tail -1 gpurun_out/${TAG}_${on}_${i}.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d.get('extra_configs',{})
print('$VAR=$on', d['value'], e.get('bf16_batch1_fps'), e.get('bf16_batch8_fps'), e.get('bf16_batch16_fps'))"
  done
done
