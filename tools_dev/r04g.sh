set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 16 > gpurun_out/r04g_ops16.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py f32 1 > gpurun_out/r04g_opsf1.txt 2>&1
MAGPIE_LIB=$PWD/ab_libs/ks4ko2.so timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -k "bf16_batch or f16_batch or sampled_batch or bf16_small or f16_small" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04g_ks_tests.log 2>&1
echo ks tests ok
MAGPIE_LIB=$PWD/ab_libs/ks4ko2.so timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 16 > gpurun_out/r04g_ops16_ks.txt 2>&1
bash tools_dev/ab_lib.sh r04g_ab 2 ab_libs/nt.so ab_libs/ks4.so ab_libs/ks8.so ab_libs/ko2.so ab_libs/ks4ko2.so > gpurun_out/r04g_ab.txt 2>&1
