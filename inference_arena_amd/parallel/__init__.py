"""Multi-GPU data parallelism: one process per GPU, RCCL over xGMI."""
