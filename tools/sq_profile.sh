#!/bin/bash
# SQ / TA counter passes (one rocprofv3 --pmc run each, no tracing) over a
# short bench run, then tools/sq_summary.py prints per-kernel issue figures.
# Usage: bash tools/sq_profile.sh <tag> [bench args...]
tag=${1:-sq}; shift
args=${@:---steps 3 --warmup 1 --no-cpu-baseline --no-csr --no-profile}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAVES" \
           "TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $out/pmc$i -o run --output-format csv -- python3 bench.py $args > $out/pmc$i.log 2>&1 || exit $?
done
python3 tools/sq_summary.py $out > $out/sq_summary.txt 2>&1 || exit $?
cat $out/sq_summary.txt
