#!/bin/bash
# PMC passes over single GraphSum configurations of tools/gs_micro.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-gsprof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P1="SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
P2="TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
P3="TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
P4="TCC_REQ_sum TCC_TAG_STALL_sum TCC_BUSY_sum TCC_EA0_RDREQ_sum"
P5="SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for cfg in d16 nogather table4096; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $P -d "$OUT/${cfg}_p$i" -o run -f csv -- python3 tools/gs_micro.py $cfg \
        > "$OUT/${cfg}_p$i.log" 2>&1 || { echo "fail $cfg $i"; exit 1; }
  done
  echo "$cfg done"
done
