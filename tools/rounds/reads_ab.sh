#!/bin/bash
# Beyond-L2 read bytes per kernel under environment settings (two PMC passes
# each: TCC_EA0_RDREQ 128B/64B/32B) plus the trace for durations.
# Usage: SETTINGS="base KR_STENCIL_Z=2" bash tools/reads_ab.sh [bench args]
export TMPDIR=/tmp
args=${@:---steps 3 --warmup 1 --no-cpu-baseline --no-csr}
for set in ${SETTINGS:-base}; do
  tag=rd_${set//[^A-Za-z0-9]/_}
  out=gpurun_out/$tag; mkdir -p $out
  envs=""; [ "$set" != base ] && envs=${set//,/ }
  export $envs 2>/dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py $args > $out/trace.log 2>&1 || exit $?
  i=0
  for pmc in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc -d $out/pmc$i -o run --output-format csv -- python3 bench.py $args --no-profile > $out/pmc$i.log 2>&1 || exit $?
  done
  [ -n "$envs" ] && for e in $envs; do unset ${e%%=*}; done
  echo "== $set"
  python3 tools/pmc_summary.py $out | grep -i "stencil" || exit $?
done
