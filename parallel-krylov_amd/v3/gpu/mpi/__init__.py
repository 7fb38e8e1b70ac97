"""One-process-per-GPU solver family (reference v3/gpu/mpi), RCCL over xGMI."""
