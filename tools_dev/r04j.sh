set -e -o pipefail
export TMPDIR=/tmp
bash tools_dev/ab_lib.sh r04j_ab 2 ab_libs/nt.so ab_libs/rw4.so ab_libs/rw1.so > gpurun_out/r04j_ab.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 16 > gpurun_out/r04j_ops16.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 8 > gpurun_out/r04j_ops8.txt 2>&1
