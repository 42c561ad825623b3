"""I/O contract, workload generation, tracing."""
