set -e -o pipefail
export TMPDIR=/tmp
bash tools_dev/ab_lib.sh r04i_ab 1 ab_libs/nt.so ab_libs/ks4.so ab_libs/ko2.so ab_libs/ks4ko2.so > gpurun_out/r04i_ab.txt 2>&1
bash tools_dev/ab_env.sh r04i_chain MAGPIE_LT_CHAIN 2 > gpurun_out/r04i_chain_ab.txt 2>&1
