set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools_dev/diag_timeline.py bf16 16 > gpurun_out/r04c_tl16.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 16 > gpurun_out/r04c_ops16.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 8 > gpurun_out/r04c_ops8.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py f32 8 > gpurun_out/r04c_opsf8.txt 2>&1
timeout -k 10 900 python -u -m pytest tests/test_decode_gpu.py tests/test_configs_gpu.py -k "batch or bf16 or f16 or sampl" -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1
echo tests ok
timeout -k 10 900 python -u -m pytest tests/test_long_range_gpu.py tests/test_xa_forms_gpu.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r04c_tests2.log 2>&1
echo tests2 ok
timeout -k 10 300 python -u tools_dev/mode_ops.py f32 1 > gpurun_out/r04c_opsf1.txt 2>&1
