#!/bin/bash
# PMC passes (MI355X_MICROARCH.md "HBM" and "rocprofv3 PMC slots"): one rocprofv3
# pass per counter group, never combined with any trace domain. FETCH_SIZE needs 3
# TCC counters and WRITE_SIZE 2, so they get separate passes; the MFMA pass holds 4
# SQ counters + 1 GRBM. Workloads: f32 B=1 decode (the bench line), bf16 B=16
# decode (configs[2]), Q8_0 B=16 decode (int8 MFMA), the codec (8 x 32 frames).
# Then tools_dev/pmc_report.py TAG.
# Usage: tools_dev/pmc_collect.sh TAG
set -e -o pipefail
TAG=${1:-r02}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp MAGPIE_EAGER=1
run() {  # name counters workload...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $ctr -f csv -d "$OUT/${TAG}_pmc_${name}" -o pmc -- python3 -u "$@" \
    > "$OUT/${TAG}_pmc_${name}.log" 2>&1
  echo "pass $name ok"
}
run f32b1_fetch FETCH_SIZE tools_dev/pmc_workload.py decode f32 1
run f32b1_write WRITE_SIZE tools_dev/pmc_workload.py decode f32 1
run b16b16_fetch FETCH_SIZE tools_dev/pmc_workload.py decode bf16 16
run b16b16_write WRITE_SIZE tools_dev/pmc_workload.py decode bf16 16
run b16b16_mfma "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
  tools_dev/pmc_workload.py decode bf16 16
run q8b16_fetch FETCH_SIZE tools_dev/pmc_workload.py decode q8 16
run q8b16_write WRITE_SIZE tools_dev/pmc_workload.py decode q8 16
run q8b16_mfma "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
  tools_dev/pmc_workload.py decode q8 16
run codec_fetch FETCH_SIZE tools_dev/pmc_workload.py codec
run codec_write WRITE_SIZE tools_dev/pmc_workload.py codec
run codec_mfma "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
  tools_dev/pmc_workload.py codec
