set -e -o pipefail
export TMPDIR=/tmp
MAGPIE_LIB=$PWD/ab_libs/lt.so timeout -k 10 900 python -u -m pytest tests/test_decode_gpu.py tests/test_long_range_gpu.py tests/test_configs_gpu.py tests/test_xa_forms_gpu.py tests/test_q8_fused_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04n_lt_tests.log 2>&1
echo pre tests ok
bash tools_dev/ab_lib.sh r04n_ab 2 ab_libs/lt.so > gpurun_out/r04n_ab.txt 2>&1
MAGPIE_LIB=$PWD/ab_libs/lt.so timeout -k 10 300 python -u tools_dev/mode_ops.py f32 1 > gpurun_out/r04n_opsf1_lt.txt 2>&1
MAGPIE_LIB=$PWD/ab_libs/lt.so timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 16 > gpurun_out/r04n_ops16_lt.txt 2>&1
