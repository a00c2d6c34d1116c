set -e -o pipefail
bash tools_dev/gpu_round.sh r04o
timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 8 > gpurun_out/r04o_ops8.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py q8 1 > gpurun_out/r04o_opsq8.txt 2>&1
