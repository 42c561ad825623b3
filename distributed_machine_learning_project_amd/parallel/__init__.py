"""Distributed strategies over torch.distributed (RCCL on MI355X, gloo on CPU)."""
