# LDS-FAR position pairs: bitwise tests, then the C4 A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out/lfar
timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py -m gpu -x -q --timeout 300 --timeout-method thread -k "position_pairs" > gpurun_out/lfar/tests.txt 2>&1; rc=$?
tail -3 gpurun_out/lfar/tests.txt
[ $rc -eq 0 ] || exit $rc
SETTINGS="base KR_STENCIL_PAIR=2 KR_STENCIL_PAIR=34 KR_STENCIL_PAIR=60 base KR_STENCIL_PAIR=34 KR_STENCIL_PAIR=60" bash tools/env_ab.sh --steps 20 --warmup 3 --no-cpu-baseline --no-csr
