#!/bin/bash
# A/B: default library vs each library given, bench (f32 B=1) + f32 parity tests
# for each. Usage: tools_dev/ab.sh TAG lib1.so [lib2.so ...]
set -e -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for L in default "$@"; do
  n=$(basename "$L" .so)
  if [ "$L" = default ]; then unset MAGPIE_LIB; else export MAGPIE_LIB=$PWD/$L; fi
  timeout -k 10 200 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "small_model_codes or full_model_codes or golden or batch_equals_single" > gpurun_out/${TAG}_${n}_t.log 2>&1
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extra --steps 5 > gpurun_out/${TAG}_${n}_b.log 2>&1
  echo "$n $(tail -1 gpurun_out/${TAG}_${n}_t.log) $(tail -1 gpurun_out/${TAG}_${n}_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], {k: v["avg_us"] for k, v in d["ops"].items()})')"
done
