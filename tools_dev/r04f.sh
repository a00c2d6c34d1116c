set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools_dev/diag_timeline.py bf16 16 qkv ff1 > gpurun_out/r04f_tl16.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 16 > gpurun_out/r04f_ops16.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py f32 1 > gpurun_out/r04f_opsf1.txt 2>&1
bash tools_dev/ab_lib.sh r04f_ab 2 ab_libs/nt.so > gpurun_out/r04f_ab.txt 2>&1
