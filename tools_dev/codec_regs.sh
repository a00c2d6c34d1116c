#!/bin/bash
# VGPR / spill / LDS / occupancy of the codec kernels for a set of -D flags.
# usage: tools_dev/codec_regs.sh "-DFOO=1 ..."
ROOT=$(cd "$(dirname "$0")/.." && pwd)
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Xclang -target-feature -Xclang -packed-fp32-ops -ffp-contract=off -Xclang -target-feature -Xclang -fma-mix-insts -Xclang -target-feature -Xclang -fma-mix-bf16-insts $1"
/opt/rocm/bin/hipcc $FLAGS --cuda-device-only -c "$ROOT/magpie-tts.cpp_amd/csrc/mp_codec.hip" -o /tmp/codec_regs.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size" \
  | sed -E 's/.*remark: //' | paste - - - - - - | grep -E "${2:-rb_kernel|conv2_kernel}" | sed -E 's/Function Name: //; s/\[-Rpass-analysis=kernel-resource-usage\]//g'
