set -e -o pipefail
export TMPDIR=/tmp
export MAGPIE_LIB=$PWD/ab_libs/probe.so
timeout -k 10 300 python -u tools_dev/diag_timeline.py bf16 16 qkv ff1 > gpurun_out/r04b_tl16.txt 2>&1
timeout -k 10 300 python -u tools_dev/diag_timeline.py bf16 8 ff1 > gpurun_out/r04b_tl8.txt 2>&1
unset MAGPIE_LIB
timeout -k 10 900 python -u -m pytest tests/test_long_range_gpu.py tests/test_decode_gpu.py tests/test_xa_forms_gpu.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1
echo tests ok
