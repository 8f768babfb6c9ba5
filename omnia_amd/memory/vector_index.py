"""Device-resident vector index: one per (workspace, embedding model).

Rows are bf16 unit vectors in a capacity-doubling matrix on the GPU (HBM is
plentiful: 10M x 1024-d = 20 GB, a fraction of one MI355X); deletes tombstone a
row (``valid`` mask consulted inside the K18 kernel) and the slot is reused.
Search = K18 cosine scores + exact radix-select top-k.  Replaces pgvector's HNSW
index (``idx_memory_observations_embedding``) with an exact scan: at ~6 TB/s a
1M x 1024 bf16 scan costs ~0.35 ms, below one HNSW probe over the network.
"""
from __future__ import annotations

import threading

import torch

from .. import ops


class VectorIndex:
    def __init__(self, dim: int, device=None, capacity: int = 1024):
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.dim = dim
        self.mat = torch.zeros(capacity, dim, dtype=torch.bfloat16, device=self.device)
        self.valid = torch.zeros(capacity, dtype=torch.uint8, device=self.device)
        self.keys: list = []
        self.row_of: dict = {}
        self.free: list[int] = []
        self._lock = threading.RLock()

    def __len__(self):
        return len(self.row_of)

    def _grow(self, need: int):
        cap = self.mat.shape[0]
        if need <= cap:
            return
        while cap < need:
            cap *= 2
        m = torch.zeros(cap, self.dim, dtype=torch.bfloat16, device=self.device)
        m[: self.mat.shape[0]] = self.mat
        v = torch.zeros(cap, dtype=torch.uint8, device=self.device)
        v[: self.valid.shape[0]] = self.valid
        self.mat, self.valid = m, v

    def upsert(self, items: list[tuple[object, list[float]]]):
        """items: (key, vector).  Vectors are normalised here."""
        if not items:
            return
        with self._lock:
            rows = []
            for key, _ in items:
                r = self.row_of.get(key)
                if r is None:
                    if self.free:
                        r = self.free.pop()
                        self.keys[r] = key
                    else:
                        r = len(self.keys)
                        self.keys.append(key)
                    self.row_of[key] = r
                rows.append(r)
            self._grow(len(self.keys))
            v = torch.tensor([x for _, x in items], dtype=torch.float32)
            if v.shape[1] != self.dim:
                raise ValueError(f"vector dim {v.shape[1]} != index dim {self.dim}")
            v = torch.nn.functional.normalize(v, dim=1)
            idx = torch.tensor(rows, dtype=torch.long, device=self.device)
            self.mat.index_copy_(0, idx, v.to(device=self.device, dtype=torch.bfloat16))
            self.valid.index_fill_(0, idx, 1)

    def remove(self, keys):
        with self._lock:
            rows = []
            for k in keys:
                r = self.row_of.pop(k, None)
                if r is not None:
                    rows.append(r)
                    self.keys[r] = None
                    self.free.append(r)
            if rows:
                self.valid.index_fill_(0, torch.tensor(rows, device=self.device), 0)

    def get(self, key):
        r = self.row_of.get(key)
        return None if r is None else self.mat[r].float().cpu()

    def search(self, queries: list[list[float]], k: int) -> list[list[tuple[object, float]]]:
        with self._lock:
            n = len(self.keys)
            if n == 0 or not self.row_of or not queries:
                return [[] for _ in queries]
            q = torch.nn.functional.normalize(torch.tensor(queries, dtype=torch.float32), dim=1)
            kk = min(k, len(self.row_of), 1024, n)
            vals, idx = ops.cosine_topk(q.to(self.device), self.mat[:n], kk, self.valid[:n])
            vals, idx = vals.cpu().tolist(), idx.cpu().tolist()
            out = []
            for vr, ir in zip(vals, idx):
                out.append([(self.keys[i], v) for v, i in zip(vr, ir)
                            if v != float("-inf") and self.keys[i] is not None])
            return out
