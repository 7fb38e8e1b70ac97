#!/bin/bash
# SQ / TA / TCP counter passes over tools/micro/csr_micro's "prof" case (the
# library's plain-CSR dual row walk and the LDS-free direct walk, 3 launches
# each), one rocprofv3 --pmc run per group. Usage: bash tools/micro/csr_pmc.sh <tag>
tag=${1:-csrpmc}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAVES" \
           "TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TD_TD_BUSY_sum TD_BUSY_avr TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d $out/pmc$i -o run --output-format csv -- tools/micro/csr_micro 512 3 prof > $out/pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/pmc$i.log; exit 1; }
done
ls -R $out | head -40
