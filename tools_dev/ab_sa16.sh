#!/bin/bash
# A/B: bf16 16 slots with the SA in the QKV launch (MAGPIE_SA16=1) vs separate, then
# the 16-slot batch tests with the knob on. Usage: tools_dev/ab_sa16.sh TAG
set -e -o pipefail
TAG=${1:-r03w}; O=gpurun_out; mkdir -p $O
for i in 1 2; do
  timeout -k 10 150 python -u tools_dev/mode_ops.py bf16 16 > $O/${TAG}_b16_16_base$i.txt 2>&1
  MAGPIE_SA16=1 timeout -k 10 150 python -u tools_dev/mode_ops.py bf16 16 > $O/${TAG}_b16_16_sa16_$i.txt 2>&1
done
MAGPIE_SA16=1 timeout -k 10 150 python -u tools_dev/mode_ops.py bf16 16 MODE_KV=bf16 > $O/${TAG}_b16kv_16_sa16.txt 2>&1
timeout -k 10 150 python -u tools_dev/mode_ops.py bf16 16 MODE_KV=bf16 > $O/${TAG}_b16kv_16_base.txt 2>&1
echo "ab ok"
MAGPIE_SA16=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_configs_gpu.py tests/test_long_range_gpu.py::test_bf16_batch16_teacher_forced_256 tests/test_kv_bf16_gpu.py \
  > $O/${TAG}_tests_sa16.log 2>&1
echo "tests ok"
