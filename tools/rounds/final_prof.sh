# Round-end rocprofv3 passes (kernel trace + PMC) of C4 and its plain-CSR run.
bash tools/profile.sh ${TAG:-r04i}_C4 > /dev/null || exit $?
tail -25 gpurun_out/${TAG:-r04i}_C4/summary.txt
KR_MASK=0 KR_VDICT=0 KR_STENCIL=0 bash tools/profile.sh ${TAG:-r04i}_C4_csr > /dev/null || exit $?
tail -12 gpurun_out/${TAG:-r04i}_C4_csr/summary.txt
