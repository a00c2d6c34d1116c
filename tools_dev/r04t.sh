set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_q8_fused_gpu.py tests/test_xa_forms_gpu.py tests/test_decode_gpu.py tests/test_configs_gpu.py -k "q8 or q4 or direct or long_text or xa" -x -v --timeout 300 --timeout-method thread > gpurun_out/r04t_tests.log 2>&1
echo tests ok
timeout -k 10 200 python -u tools_dev/diag_handoff_q8.py 3 1 > gpurun_out/r04t_handoff_q8.txt 2>&1
timeout -k 10 200 python -u tools_dev/mode_ops.py q8 1 q8 > gpurun_out/r04t_ops_q8_b1.txt 2>&1
timeout -k 10 200 python -u tools_dev/mode_ops.py q8 8 q8 > gpurun_out/r04t_ops_q8_b8.txt 2>&1
timeout -k 10 200 python -u tools_dev/diag_timeline.py f32 1 > gpurun_out/r04t_timeline_f32_b1.txt 2>&1
echo diag ok
