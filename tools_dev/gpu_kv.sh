#!/bin/bash
# bf16-KV + decode GPU tests, then the codec trace
set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kv_bf16_gpu.py tests/test_decode_gpu.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/kv_tests.log 2>&1 || { tail -40 gpurun_out/kv_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/kv_tests.log | tail -2
grep -E "bf16 KV|prefill K/V|teacher-forced" gpurun_out/kv_tests.log | head -8 || true
