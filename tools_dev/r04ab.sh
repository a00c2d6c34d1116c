set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_q8_fused_gpu.py tests/test_long_range_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ab_tests.log 2>&1
echo tests ok
bash tools_dev/ab_lib.sh r04ab_ab 2 ab_libs/base.so > gpurun_out/r04ab_ab.txt 2>&1
echo ab ok
timeout -k 10 200 python -u tools_dev/mode_ops.py f32 1 > gpurun_out/r04ab_ops_f32_b1.txt 2>&1
echo ops ok
