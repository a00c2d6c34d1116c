#!/bin/bash
# Per-op A/B of library builds on one box: ab_ops.sh OUTPREFIX DIR... (DIR/lib/libmagpie_hip.so)
set -e -o pipefail
P=$1; shift
for R in 1 2; do
  for D in "$@"; do
    n=$(basename "$D")
    MAGPIE_LIB=$D/lib/libmagpie_hip.so timeout -k 10 200 python bench.py --steps 3 --no-codec --no-cpu-baseline --no-extra > gpurun_out/${P}_${n}_$R.json 2> gpurun_out/${P}_${n}_$R.err
  done
done
