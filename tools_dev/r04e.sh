set -e -o pipefail
export TMPDIR=/tmp
export MAGPIE_LIB=$PWD/ab_libs/probe.so
timeout -k 10 300 python -u tools_dev/probe_report.py bf16 16 qkv ff1 > gpurun_out/r04e_probe16.txt 2>&1
timeout -k 10 300 python -u tools_dev/probe_report.py bf16 8 ff1 > gpurun_out/r04e_probe8.txt 2>&1
timeout -k 10 300 python -u tools_dev/probe_report.py f32 8 ff1 qkv_sa > gpurun_out/r04e_probef8.txt 2>&1
