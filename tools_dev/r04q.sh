set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_q8_fused_gpu.py tests/test_decode_gpu.py tests/test_configs_gpu.py -k "q8 or q4" -x -v --timeout 300 --timeout-method thread > gpurun_out/r04q_tests.log 2>&1
echo q8 tests ok
for i in 1 2; do
  for m in 0 2; do
    timeout -k 10 200 python -u tools_dev/mode_ops.py q8 1 q8 MAGPIE_LTQ8=$m > gpurun_out/r04q_ops_q8_m${m}_$i.txt 2>&1
    head -3 gpurun_out/r04q_ops_q8_m${m}_$i.txt | grep frames
  done
done
timeout -k 10 200 python -u tools_dev/mode_ops.py q8 16 q8 > gpurun_out/r04q_ops_q8_b16.txt 2>&1
head -3 gpurun_out/r04q_ops_q8_b16.txt | grep frames
timeout -k 10 200 python -u tools_dev/diag_handoff_q8.py 3 1 > gpurun_out/r04q_handoff_q8.txt 2>&1
echo diag ok
