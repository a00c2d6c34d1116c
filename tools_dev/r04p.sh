set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_configs_gpu.py tests/test_q8_fused_gpu.py -k "f16 or q8 or q4" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04p_q8f16_tests.log 2>&1
echo q8/f16 tests ok
bash tools_dev/ab_lib.sh r04p_ab 2 ab_libs/lts16.so > gpurun_out/r04p_ab.txt 2>&1
MAGPIE_LIB=$PWD/ab_libs/lts16.so timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py tests/test_configs_gpu.py tests/test_long_range_gpu.py -k "bf16" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04p_lts16_tests.log 2>&1
echo lts16 tests ok
bash tools_dev/pmc_collect.sh r04p > gpurun_out/r04p_pmc.log 2>&1
echo pmc ok
