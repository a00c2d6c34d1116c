#!/bin/bash
# A/B of library builds on one box: bench (f32 B=1 + the bf16 batch extras) with the
# default library and each given ab_libs/*.so, alternating, N rounds.
# usage: tools_dev/ab_lib.sh TAG N lib.so [lib.so ...]
set -e -o pipefail
TAG=$1; N=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for L in default "$@"; do
    n=$(basename "$L" .so)
    if [ "$L" = default ]; then unset MAGPIE_LIB; else export MAGPIE_LIB=$PWD/$L; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-codec --steps 10 > gpurun_out/${TAG}_${n}_${i}.log 2>&1
    tail -1 gpurun_out/${TAG}_${n}_${i}.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d.get('extra_configs',{})
print('$n', round(d['value'],1), e.get('bf16_batch1_fps'), e.get('bf16_batch8_fps'), e.get('bf16_batch16_fps'), e.get('q8_batch1_fps'))"
  done
done
