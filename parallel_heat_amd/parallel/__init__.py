"""Decomposition and inter-rank plumbing (one process per GPU, torch.distributed + RCCL)."""
from .topology import Block, Cart, block_span, dims_create, layout, memory_plan
from .comm import (DistInfo, LoopbackHub, TorchDistTransport, env_info, init_distributed,
                   make_comm)
# parallel.group (threads over the loopback transport) imports the model
# layer; import it explicitly: `from parallel_heat_amd.parallel.group import run_group`.

__all__ = ["Block", "Cart", "block_span", "dims_create", "layout", "memory_plan", "DistInfo",
           "LoopbackHub", "TorchDistTransport", "env_info", "init_distributed", "make_comm"]
