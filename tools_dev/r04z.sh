set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_q8_fused_gpu.py tests/test_long_range_gpu.py tests/test_xa_forms_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04z_tests.log 2>&1
echo tests ok
bash tools_dev/ab_lib.sh r04z_ab 2 ab_libs/base.so ab_libs/gap16.so ab_libs/gap2.so > gpurun_out/r04z_ab.txt 2>&1
echo ab ok
