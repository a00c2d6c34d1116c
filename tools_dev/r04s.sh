set -e -o pipefail
export TMPDIR=/tmp
bash tools_dev/ab_envs.sh r04s_env 2 - HIP_FORCE_DEV_KERNARG=1 HIP_FORCE_DEV_KERNARG=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 > gpurun_out/r04s_env.txt 2>&1
echo env ok
timeout -k 10 200 python -u tools_dev/diag_timeline.py bf16 8 > gpurun_out/r04s_timeline_bf16_b8.txt 2>&1
echo timeline ok
