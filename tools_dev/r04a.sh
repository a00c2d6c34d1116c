set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools_dev/diag_timeline.py bf16 16 > gpurun_out/r04a_tl16.txt 2>&1
timeout -k 10 300 python -u tools_dev/diag_timeline.py bf16 8 > gpurun_out/r04a_tl8.txt 2>&1
timeout -k 10 300 python -u tools_dev/mode_ops.py bf16 16 > gpurun_out/r04a_ops16.txt 2>&1
echo done
