# Same-box A/B of the stencil code patterns (KR_STENCIL_PATTERNS=0: per-row code stream).
SETTINGS="base KR_STENCIL_PATTERNS=0 base KR_STENCIL_PATTERNS=0" bash tools/env_ab.sh --steps 20 --warmup 3 --no-cpu-baseline --no-csr || exit $?
SETTINGS="base KR_STENCIL_PATTERNS=0 base KR_STENCIL_PATTERNS=0" bash tools/env_ab.sh --config C2 --steps 300 --warmup 20 --no-cpu-baseline
