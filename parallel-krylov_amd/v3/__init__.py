"""Mirror of the reference's v3 API generation (5enxia/parallel-krylov v3/)."""
