set -e -o pipefail
export TMPDIR=/tmp
PHASES=1 timeout -k 10 200 python -u tools_dev/diag_timeline.py bf16 8 qkv_sa oproj_xa > gpurun_out/r04ad_tl_bf16_b8.txt 2>&1
PHASES=1 timeout -k 10 200 python -u tools_dev/diag_timeline.py bf16 1 qkv_sa oproj_xa > gpurun_out/r04ad_tl_bf16_b1.txt 2>&1
PHASES=1 timeout -k 10 200 python -u tools_dev/diag_timeline.py f32 1 qkv_sa oproj_xa > gpurun_out/r04ad_tl_f32_b1.txt 2>&1
echo ok
