# PMC passes of C3 and C5 after the DIA walk's full-block run (no mask loads).
bash tools/profile.sh ${TAG:-r04m}_C3 --config C3 --steps 20 --warmup 2 --no-cpu-baseline --no-csr > /dev/null || exit $?
bash tools/profile.sh ${TAG:-r04m}_C5 --config C5 --steps 2 --warmup 1 --no-cpu-baseline --no-csr > /dev/null || exit $?
for c in C3 C5; do echo "== $c"; grep -E "spmv|update" gpurun_out/${TAG:-r04m}_$c/summary.txt | head -12; done
