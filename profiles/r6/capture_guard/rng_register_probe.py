"""Probe: does a graph capture allocate default-pool blocks when no other graph
is alive (PyTorch's generator graph-state registration)?"""
import gc

import torch

from omnia_amd.engine.capture_guard import _active_default_blocks

dev = torch.device("cuda", 0)
pool = torch.cuda.graph_pool_handle()
x = torch.zeros(16, device=dev)


def capture():
    g = torch.cuda.CUDAGraph()
    before = _active_default_blocks(dev)
    with torch.cuda.graph(g, pool=pool):
        x.add_(1)
    return g, sorted(_active_default_blocks(dev) - before)


g1, new1 = capture()
print("first capture, no graph alive:", new1)
g2, new2 = capture()
print("second capture, g1 alive:", new2)
del g1, g2
gc.collect()
g3, new3 = capture()
print("after every graph was dropped:", new3)
