set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_long_range_gpu.py tests/test_configs_gpu.py -k "bf16 or f16 or batch" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04x_tests.log 2>&1
echo tests ok
bash tools_dev/ab_lib.sh r04x_ab 2 ab_libs/base.so > gpurun_out/r04x_ab.txt 2>&1
echo ab ok
