set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_q8_fused_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04v_tests.log 2>&1
echo tests ok
timeout -k 10 200 python -u tools_dev/diag_handoff_q8.py 3 1 > gpurun_out/r04v_handoff_q8.txt 2>&1
timeout -k 10 200 python -u tools_dev/mode_ops.py q8 1 q8 > gpurun_out/r04v_ops_q8_b1.txt 2>&1
echo diag ok
