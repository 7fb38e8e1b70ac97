#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then PMC
# passes (one counter group per pass; never combined with tracing domains).
# Usage: bash tools/profile.sh <tag> [bench args...]
tag=${1:-prof}; shift
args=${@:---steps 5 --warmup 1 --no-cpu-baseline}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT 2>/dev/null || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py $args > $out/trace.log 2>&1 || exit $?
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $pmc | tr ' ' '_')
  timeout -k 10 600 rocprofv3 --pmc $pmc -d $out/pmc_$name -o run --output-format csv -- python3 bench.py $args --no-profile > $out/pmc_$name.log 2>&1 || exit $?
done
echo done
