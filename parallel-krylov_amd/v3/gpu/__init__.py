"""Single-process GPU solver family (reference v3/gpu), on libkrylov_amd."""
