set -e -o pipefail
export TMPDIR=/tmp
MAGPIE_LT_CHAIN=1 timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_long_range_gpu.py tests/test_cli_gpu.py -k "not bf16 and not f16 and not q8 and not q4" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04h_chain_tests.log 2>&1
echo chain tests ok
MAGPIE_LT_CHAIN=2 timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_long_range_gpu.py -k "not bf16 and not f16 and not q8 and not q4 and not 500" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04h_chain2_tests.log 2>&1
echo chain2 tests ok
MAGPIE_LT_CHAIN=2 timeout -k 10 300 python -u tools_dev/mode_ops.py f32 1 > gpurun_out/r04h_opsf1_chain2.txt 2>&1
MAGPIE_LT_CHAIN=1 timeout -k 10 300 python -u tools_dev/mode_ops.py f32 1 > gpurun_out/r04h_opsf1.txt 2>&1
MAGPIE_LT_CHAIN=0 timeout -k 10 300 python -u tools_dev/mode_ops.py f32 1 > gpurun_out/r04h_opsf1_nochain.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 16 > gpurun_out/r04h_ops16.txt 2>&1
MAGPIE_LIB=$PWD/ab_libs/ks4ko2.so timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -k "bf16_batch or f16_batch or sampled_batch or bf16_small or f16_small" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04h_ks_tests.log 2>&1
echo ks tests ok
MAGPIE_LIB=$PWD/ab_libs/ks4ko2.so timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 16 > gpurun_out/r04h_ops16_ks.txt 2>&1
