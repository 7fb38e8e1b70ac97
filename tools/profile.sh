#!/bin/bash
# rocprofv3 passes over one short bench run (GPU box):
#   1. --kernel-trace --stats            (durations; never combined with PMC)
#   2.. one PMC group per pass            (TCC slots are scarce; separate runs)
# then tools/pmc_summary.py writes gpurun_out/<tag>/summary.json.
# Usage: bash tools/profile.sh <tag> [bench args...]
# One config per call (kernel names must be unique per profile): the bench
# args default to the C4 headline without its plain-CSR sub-run; profile the
# CSR format with `KR_MASK=0 KR_VDICT=0 KR_STENCIL=0 bash tools/profile.sh <tag>`.
tag=${1:-prof}; shift
args=${@:---steps 5 --warmup 1 --no-cpu-baseline --no-csr}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py $args > $out/trace.log 2>&1 || exit $?
i=0
for pmc in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $pmc -d $out/pmc$i -o run --output-format csv -- python3 bench.py $args --no-profile > $out/pmc$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $out > $out/summary.txt 2>&1 || exit $?
cat $out/summary.txt
