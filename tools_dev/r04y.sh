set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04y_tests.log 2>&1
echo tests ok
bash tools_dev/ab_lib.sh r04y_ab 2 ab_libs/base.so > gpurun_out/r04y_ab.txt 2>&1
echo ab ok
