#!/bin/bash
# A/B of two builds on one box: ab_bench.sh DIR_A DIR_B [frames] [batches...]
# DIR_x holds bin/mp_bench + lib/libmagpie_hip.so (rpath $ORIGIN/../lib).
set -e -o pipefail
C=${MAGPIE_CACHE:-/tmp/magpie_amd_cache}; mkdir -p "$C"
M="$C/magpie_full.gguf"
[ -f "$M" ] || magpie-tts.cpp_amd/bin/mp_synth_gguf magpie "$M" >/dev/null
A=$1; B=$2; F=${3:-256}; shift 3 || true
for NB in ${@:-1 8}; do
  for R in 1 2; do
    for D in "$A" "$B"; do
      echo "== $D batch $NB"
      timeout -k 10 120 "$D/bin/mp_bench" "$M" "$F" "$NB" 2 64 | tail -1
    done
  done
done
