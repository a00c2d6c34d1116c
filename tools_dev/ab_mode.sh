#!/bin/bash
# A/B of per-op launch times: tools_dev/ab_mode.sh TAG "WEIGHTS B [args]" [lib.so ...]
# (default library first, then each given library; tools_dev/mode_ops.py per library)
set -e -o pipefail
TAG=$1; MODE=$2; shift 2
mkdir -p gpurun_out
for L in default "$@"; do
  n=$(basename "$L" .so)
  if [ "$L" = default ]; then unset MAGPIE_LIB; else export MAGPIE_LIB=$PWD/$L; fi
  timeout -k 10 150 python -u tools_dev/mode_ops.py $MODE > gpurun_out/${TAG}_${n}.txt 2>&1
  echo "$n $(head -1 gpurun_out/${TAG}_${n}.txt)"
done
