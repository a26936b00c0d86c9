"""Probe: can two processes drive RCCL communicators on the same GPU?"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
from parallel_heat_amd import HeatConfig, HeatSolver
from parallel_heat_amd.parallel.comm import DistInfo
cfg = HeatConfig(nx=256, ny=512, steps=0, init="random", backend="hip", tb_depth=8, device=0)
t = time.time()
try:
    s = HeatSolver(cfg, transport="rccl", dist_info=DistInfo(rank, world, 0), device=0)
    r = s.run(64)
    g = s.gather()
    if rank == 0:
        ref = HeatSolver(cfg, transport="local", dist_info=DistInfo(0, 1, 0), device=0)
        ref.run(64)
        print("RCCL same-device OK, equal:", __import__("numpy").array_equal(g, ref.gather()), "time", time.time() - t, flush=True)
    s.close()
    print(f"rank {rank} ok", flush=True)
except Exception as e:
    print(f"rank {rank} RCCL same-device FAILED: {e}", flush=True)
