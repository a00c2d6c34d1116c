#!/bin/bash
# One GPU call: GPU parity tests, the default bench line, and a rocprofv3
# kernel-trace summary of the same bench (eager launches so every kernel is
# traced individually).  Usage: tools_dev/gpu_round.sh TAG [skip-tests]
# Outputs go to gpurun_out/TAG_*.  Every GPU step has its own time limit and
# the chain stops at the first failure.
set -e -o pipefail
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread \
    > "$OUT/${TAG}_gpu_tests.log" 2>&1
  echo "gpu tests ok"
fi
timeout -k 10 300 python -u bench.py > "$OUT/${TAG}_bench.log" 2>&1
tail -1 "$OUT/${TAG}_bench.log" > "$OUT/${TAG}_bench.json"
echo "bench ok"
MAGPIE_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_prof" -o prof \
  -- python3 -u bench.py --no-cpu-baseline --no-extra > "$OUT/${TAG}_prof_bench.log" 2>&1
python3 tools_dev/prof_phase.py "$OUT/${TAG}_prof/prof_kernel_trace.csv" "$OUT/${TAG}_prof/phase_kernel_stats.csv" \
  > "$OUT/${TAG}_prof_phase.log"
echo "rocprof ok"
