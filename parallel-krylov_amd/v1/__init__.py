"""Mirror of the reference's v1 API generation, for the one v1 component on
SURVEY.md §8(f): the preconditioned / pipelined CG variants of
v1/threads/pipeline (the rest of v1 is superseded by v3)."""
