#!/bin/bash
# Native batched-decode sweep on the GPU box: bench_batch.sh [frames] [batches...]
set -e -o pipefail
C=${MAGPIE_CACHE:-/tmp/magpie_amd_cache}; mkdir -p "$C"
M="$C/magpie_full.gguf"
[ -f "$M" ] || magpie-tts.cpp_amd/bin/mp_synth_gguf magpie "$M" >/dev/null
F=${1:-256}; shift || true
for B in ${@:-1 2 4 8}; do
  timeout -k 10 120 magpie-tts.cpp_amd/bin/mp_bench "$M" "$F" "$B" 2 64
done
