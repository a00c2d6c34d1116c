set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_q8_fused_gpu.py tests/test_decode_gpu.py tests/test_configs_gpu.py -k "q8 or q4" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ah_tests.log 2>&1
echo tests ok
for i in 1 2; do
  for B in 1 8; do
    MAGPIE_LIB=$PWD/ab_libs/base.so timeout -k 10 200 python -u tools_dev/mode_ops.py q8 $B q8 > gpurun_out/r04ah_base_${B}_$i.txt 2>&1
    timeout -k 10 200 python -u tools_dev/mode_ops.py q8 $B q8 > gpurun_out/r04ah_new_${B}_$i.txt 2>&1
  done
done
grep -H frames gpurun_out/r04ah_*_1_*.txt gpurun_out/r04ah_*_8_*.txt
