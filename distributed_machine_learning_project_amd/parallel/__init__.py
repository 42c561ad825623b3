"""Distributed strategies over torch.distributed (RCCL on MI355X, gloo on CPU)."""
from .comm import Comm, block_partition, dims_create  # noqa: F401
from .engine import Engine, KNNOutput  # noqa: F401
from .strategies import STRATEGIES  # noqa: F401
