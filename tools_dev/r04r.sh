set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_q8_fused_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04r_tests.log 2>&1
echo q8 tests ok
timeout -k 10 200 python -u tools_dev/diag_handoff_q8.py 3 1 > gpurun_out/r04r_handoff_q8.txt 2>&1
for m in 2 0 1; do
  timeout -k 10 200 python -u tools_dev/mode_ops.py q8 16 q8 MAGPIE_LTQ8=$m > gpurun_out/r04r_ops_q8_b16_m$m.txt 2>&1
done
timeout -k 10 200 python -u tools_dev/mode_ops.py q8 8 q8 > gpurun_out/r04r_ops_q8_b8.txt 2>&1
timeout -k 10 200 python -u tools_dev/mode_ops.py q8 4 q8 > gpurun_out/r04r_ops_q8_b4.txt 2>&1
timeout -k 10 200 python -u tools_dev/mode_ops.py q8 4 q8 MAGPIE_LTQ8=0 > gpurun_out/r04r_ops_q8_b4_m0.txt 2>&1
timeout -k 10 200 python -u tools_dev/mode_ops.py q8 1 q8 > gpurun_out/r04r_ops_q8_b1.txt 2>&1
echo ops ok
