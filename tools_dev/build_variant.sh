#!/bin/bash
# Build a variant of libmagpie_hip.so with extra compile flags into ab_libs/NAME.so
# (A/B runs select it with MAGPIE_LIB). usage: tools_dev/build_variant.sh NAME "-DFOO=1 ..."
set -e -o pipefail
NAME=$1; EXTRA=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/magpie-tts.cpp_amd
OUT=$ROOT/ab_libs/$NAME
mkdir -p "$OUT"
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -Wno-unused-value -Xclang -target-feature -Xclang -packed-fp32-ops -ffp-contract=off -Xclang -target-feature -Xclang -fma-mix-insts -Xclang -target-feature -Xclang -fma-mix-bf16-insts $EXTRA"
pids=()
for s in mp_decode mp_decode_b16 mp_decode_q8 mp_prefill mp_runtime mp_codec; do
  /opt/rocm/bin/hipcc $FLAGS -c "$PKG/csrc/$s.hip" -o "$OUT/$s.o" & pids+=($!)
done
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -Wall -c "$PKG/csrc/magpie_api.cpp" -o "$OUT/magpie_api.o" & pids+=($!)
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -Wall -c "$PKG/csrc/mp_tokenizer.cpp" -o "$OUT/mp_tokenizer.o" & pids+=($!)
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc $FLAGS -shared -Wl,-rpath,/opt/rocm/lib -o "$ROOT/ab_libs/$NAME.so" "$OUT"/*.o
echo "built ab_libs/$NAME.so"
