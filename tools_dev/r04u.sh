set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python -u tools_dev/diag_handoff_q8.py 3 1 > gpurun_out/r04u_handoff_q8.txt 2>&1
echo diag ok
