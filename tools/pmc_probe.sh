#!/bin/bash
# dev: PMC passes over the conv3w probe builds (cycles and stall counters per dispatch, no stamps)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && OUT=gpurun_out/${1:-pmcp} && mkdir -p $OUT &&
A="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
B="SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
for spec in "ns:0" "ns_a1:0" "ns_a4:0" "ns:1" "ns:0:1"; do
  IFS=: read v z var <<< "$spec"
  n=${v}_z${z}_v${var:-0}
  for p in A B; do
    timeout -s KILL 60 rocprofv3 --pmc ${!p} --output-format csv -d $OUT/$n$p -o run -- tools/conv3w_probe_$v 130 46 82 128 128 10 1 $z ${var:-0} > $OUT/$n$p.log 2>&1 || exit 1
  done
done
