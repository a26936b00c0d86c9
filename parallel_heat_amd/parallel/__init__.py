"""Decomposition and inter-rank plumbing (one process per GPU, torch.distributed + RCCL)."""
from .topology import Block, Cart, block_span, dims_create, layout, memory_plan
from .comm import DistInfo, TorchDistTransport, env_info, init_distributed, make_comm

__all__ = ["Block", "Cart", "block_span", "dims_create", "layout", "memory_plan", "DistInfo",
           "TorchDistTransport", "env_info", "init_distributed", "make_comm"]
