#!/bin/bash
# codec GPU tests + per-dispatch kernel trace of the last decode (tools_dev/codec_trace_report.py)
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-ct}
timeout -k 10 200 python -u -m pytest tests/test_codec_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 100 rocprofv3 --kernel-trace -d gpurun_out/$TAG -o ct --output-format csv -- python tools_dev/codec_prof.py > gpurun_out/$TAG.log 2>&1
python tools_dev/codec_trace_report.py $(find gpurun_out/$TAG -name "*kernel_trace.csv")
