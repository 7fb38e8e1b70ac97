# rocprofv3 trace + PMC passes of C2, C3 and C5 at the final kernels.
bash tools/profile.sh ${TAG:-r04l}_C2 --config C2 --steps 20 --warmup 2 --no-cpu-baseline --no-csr > /dev/null || exit $?
bash tools/profile.sh ${TAG:-r04l}_C3 --config C3 --steps 20 --warmup 2 --no-cpu-baseline --no-csr > /dev/null || exit $?
bash tools/profile.sh ${TAG:-r04l}_C5 --config C5 --steps 2 --warmup 1 --no-cpu-baseline --no-csr > /dev/null || exit $?
for c in C2 C3 C5; do echo "== $c"; grep -E "spmv|update" gpurun_out/${TAG:-r04l}_$c/summary.txt | head -12; done
