set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools_dev/diag_timeline.py bf16 16 > gpurun_out/r04d_tl16.txt 2>&1
timeout -k 10 300 python -u tools_dev/diag_timeline.py f32 1 > gpurun_out/r04d_tlf1.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 16 > gpurun_out/r04d_ops16.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py f32 1 > gpurun_out/r04d_opsf1.txt 2>&1
timeout -k 10 900 python -u -m pytest tests/test_decode_gpu.py tests/test_configs_gpu.py tests/test_long_range_gpu.py tests/test_xa_forms_gpu.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1
echo tests ok
