#!/bin/bash
# SQ / TCC counter passes over the codec workload (tools_dev/codec_prof.py, eager),
# one rocprofv3 --pmc pass per group, then a per-dispatch table of the last decode.
set -e -o pipefail
OUT=gpurun_out/cpmc
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr -f csv -d $OUT/p$i -o pmc -- python3 -u tools_dev/codec_prof.py > $OUT/p$i.log 2>&1
  echo "pass $i ok"
done
python3 tools_dev/codec_pmc_report.py $OUT > $OUT/report.txt
