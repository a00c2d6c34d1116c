set -e -o pipefail
export TMPDIR=/tmp
bash tools_dev/ab_lib.sh r04af_ab 2 ab_libs/sad24.so ab_libs/sad64.so > gpurun_out/r04af_ab.txt 2>&1
echo ab ok
