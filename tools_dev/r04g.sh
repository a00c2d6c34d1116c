set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools_dev/diag_timeline.py bf16 16 qkv ff1 ff2 > gpurun_out/r04g_tl16.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 16 > gpurun_out/r04g_ops16.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py f32 1 > gpurun_out/r04g_opsf1.txt 2>&1
MAGPIE_LIB=$PWD/ab_libs/ks4.so timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -k "bf16_batch or f16_batch or sampled_batch" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04g_ks4_tests.log 2>&1
echo ks4 tests ok
bash tools_dev/ab_lib.sh r04g_ab 2 ab_libs/nt.so ab_libs/ks4.so ab_libs/ks2.so > gpurun_out/r04g_ab.txt 2>&1
