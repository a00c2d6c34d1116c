set -e -o pipefail
export TMPDIR=/tmp
MAGPIE_LIB=$PWD/ab_libs/probe.so timeout -k 10 200 python -u tools_dev/probe_report.py bf16 8 qkv_sa ff1 > gpurun_out/r04w_probe_bf16_b8.txt 2>&1
MAGPIE_LIB=$PWD/ab_libs/probe.so timeout -k 10 200 python -u tools_dev/probe_report.py bf16 1 qkv_sa ff1 > gpurun_out/r04w_probe_bf16_b1.txt 2>&1
timeout -k 10 200 python -u tools_dev/mode_ops.py bf16 8 > gpurun_out/r04w_ops_bf16_b8.txt 2>&1
timeout -k 10 200 python -u tools_dev/mode_ops.py bf16 1 > gpurun_out/r04w_ops_bf16_b1.txt 2>&1
timeout -k 10 200 python -u tools_dev/diag_timeline.py bf16 1 > gpurun_out/r04w_timeline_bf16_b1.txt 2>&1
echo ok
