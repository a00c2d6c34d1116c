set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_q8_fused_gpu.py tests/test_long_range_gpu.py tests/test_configs_gpu.py tests/test_xa_forms_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ae_tests.log 2>&1
echo tests ok
bash tools_dev/ab_lib.sh r04ae_ab 2 ab_libs/base.so > gpurun_out/r04ae_ab.txt 2>&1
echo ab ok
for i in 1 2; do
  MAGPIE_LIB=$PWD/ab_libs/base.so timeout -k 10 200 python -u tools_dev/mode_ops.py q8 8 q8 > gpurun_out/r04ae_q8b8_base_$i.txt 2>&1
  timeout -k 10 200 python -u tools_dev/mode_ops.py q8 8 q8 > gpurun_out/r04ae_q8b8_new_$i.txt 2>&1
done
grep -h frames gpurun_out/r04ae_q8b8_*
