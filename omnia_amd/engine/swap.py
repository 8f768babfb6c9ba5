"""Warm KV tier: evicted session pages parked in pinned host DRAM.

Copies run on a dedicated HIP stream so they overlap the engine's compute
stream; swap-in synchronises that stream before the pages are used.
"""
from __future__ import annotations

from collections import OrderedDict

import torch


class SwapSpace:
    def __init__(self, kv, gib: float):
        self.kv = kv
        k0 = kv.k[0]
        self.page_shape = k0.shape[1:]  # [Hkv, BS, D]
        self.page_bytes = 2 * len(kv.k) * k0[0].numel() * k0.element_size()
        self.capacity_pages = int(gib * 2**30) // max(1, self.page_bytes)
        self.used = 0
        self.parked: "OrderedDict[str, object]" = OrderedDict()
        self.stream = torch.cuda.Stream() if k0.is_cuda else None

    def can_hold(self, n_pages: int) -> bool:
        while self.used + n_pages > self.capacity_pages and self.parked:
            _, s = self.parked.popitem(last=False)
            self.drop(s.swapped)
        return self.used + n_pages <= self.capacity_pages

    def swap_out(self, blocks: list[int]):
        idx = torch.tensor(blocks, device=self.kv.k[0].device)
        L = len(self.kv.k)
        host = torch.empty((L, 2, len(blocks), *self.page_shape), dtype=self.kv.k[0].dtype,
                           pin_memory=self.stream is not None)
        if self.stream is not None:
            self.stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.stream):
                for l in range(L):
                    host[l, 0].copy_(self.kv.k[l].index_select(0, idx), non_blocking=True)
                    host[l, 1].copy_(self.kv.v[l].index_select(0, idx), non_blocking=True)
            # freed pages may be reused by the next step: order it after the copy-out
            torch.cuda.current_stream().wait_stream(self.stream)
        else:
            for l in range(L):
                host[l, 0].copy_(self.kv.k[l].index_select(0, idx))
                host[l, 1].copy_(self.kv.v[l].index_select(0, idx))
        self.used += len(blocks)
        return host

    def swap_in(self, host, blocks: list[int]):
        idx = torch.tensor(blocks, device=self.kv.k[0].device)
        if self.stream is not None:
            self.stream.synchronize()
        for l in range(len(self.kv.k)):
            self.kv.k[l].index_copy_(0, idx, host[l, 0].to(self.kv.k[l].device, non_blocking=True))
            self.kv.v[l].index_copy_(0, idx, host[l, 1].to(self.kv.v[l].device, non_blocking=True))
        self.used -= host.shape[2]

    def drop(self, host):
        if host is not None:
            self.used -= host.shape[2]

    def park(self, sid, s):
        self.parked[sid] = s

    def unpark(self, sid):
        return self.parked.pop(sid, None)

    def has(self, sid) -> bool:
        return sid in self.parked
