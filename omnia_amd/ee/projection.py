"""Memory Galaxy projection: a stable 2-D layout of a workspace's memories,
rendered in the background and served from the store.

Parity map (behaviour only):

* pipeline basis -> vectorise -> reduce -> t-SNE -> Procrustes -> normalise --
  ``ee/pkg/memory/projection/project.go``
* lexical basis (TF-IDF + truncated SVD) -- ``projection/tfidf.go``; dense basis
  (PCA to 50 dims) -- ``projection/pca.go``; t-SNE -- ``projection/tsne.go``;
  Procrustes alignment to the previous layout -- ``projection/procrustes.go``
* fingerprint + render decision (unchanged / change threshold / cron) --
  ``projection/fingerprint.go``, ``ee/pkg/memory/projectionworker/schedule.go``
* render worker (policy ``spec.projection``, workspace lock, metrics) --
  ``projectionworker/worker.go``, ``metrics.go``
* defaults (cap 2000, dense threshold 0.7, 50 PCA/LSA dims, tiny set 30,
  preview 120) -- ``internal/memory/projection``

MI355X-first: every stage is a dense tensor op on the device that holds the
vector index. Exact t-SNE is O(n^2) per iteration, which at the 2,000-point
cap is a 4M-element elementwise pass plus an [n, n] x [n, 2] GEMM -- a few
microseconds of HBM traffic on the GPU -- so there is no Barnes-Hut
approximation and no host round trip inside the 1,000 iterations. The
perplexity calibration is a vectorised bisection over all rows at once.
"""
from __future__ import annotations

import json
import logging
import math
import re
import time
from dataclasses import dataclass

from ..observability import metrics as _m
from ..utils import cron

log = logging.getLogger("omnia.memory.projection")

BASIS_DENSE, BASIS_LEXICAL, BASIS_UNKNOWN = "dense", "lexical", "unknown"
MODEL_TSNE, MODEL_PCA = "tsne", "pca"

RENDERS = _m.Counter("omnia_memory_projection_renders_total", "Projection renders",
                     ["workspace", "policy", "status", "basis"], registry=_m.REGISTRY)
RENDER_SECONDS = _m.Histogram("omnia_memory_projection_render_seconds",
                              "Projection render wall time", ["workspace", "policy"],
                              registry=_m.REGISTRY)


@dataclass
class Options:
    cap: int = 2000
    dense_threshold: float = 0.7
    pca_dims: int = 50
    lsa_dims: int = 50
    preview_chars: int = 120
    tiny_set: int = 30
    tsne_iters: int = 1000
    seed: int = 0


@dataclass
class Input:
    entity_id: str
    content: str
    embedding: object  # 1-D float array or None
    tier: str = ""
    kind: str = ""
    user: str = ""
    category: str = ""
    confidence: float = 0.0
    title: str = ""
    observed_at: float = 0.0
    expires_at: float | None = None


def _device(device=None):
    import torch

    if device is not None:
        return torch.device(device)
    return torch.device("cuda" if torch.cuda.is_available() else "cpu")


# ------------------------------------------------------------------ stages
def choose_basis(inputs: list[Input], threshold: float) -> str:
    if not inputs:
        return BASIS_LEXICAL
    with_emb = sum(1 for i in inputs if i.embedding is not None and len(i.embedding))
    return BASIS_DENSE if with_emb / len(inputs) >= threshold else BASIS_LEXICAL


def select_inputs(inputs: list[Input], basis: str) -> tuple[list[Input], int]:
    if basis == BASIS_LEXICAL:
        return list(inputs), 0
    used = [i for i in inputs if i.embedding is not None and len(i.embedding)]
    return used, len(inputs) - len(used)


def apply_cap(inputs: list[Input], cap: int) -> tuple[list[Input], bool]:
    if len(inputs) <= cap:
        return inputs, False
    s = sorted(inputs, key=lambda i: (-i.observed_at, -i.confidence))
    return s[:cap], True


_TOKEN = re.compile(r"[a-z0-9]+")


def tokenize(s: str) -> list[str]:
    return [t for t in _TOKEN.findall((s or "").lower()) if len(t) > 2]


def tfidf_lsa(docs: list[str], dims: int, device=None):
    """TF-IDF (tf = count/len, idf = ln((n+1)/(df+1))) then the top-``dims``
    left singular directions scaled by their singular values."""
    import torch

    toks = [tokenize(d) for d in docs]
    df: dict = {}
    for t in toks:
        for w in set(t):
            df[w] = df.get(w, 0) + 1
    vocab = sorted(df)
    dev = _device(device)
    if not vocab:
        return torch.zeros(len(docs), 1, device=dev)
    idx = {w: i for i, w in enumerate(vocab)}
    n = len(docs)
    rows, cols, vals = [], [], []
    for r, t in enumerate(toks):
        if not t:
            continue
        counts: dict = {}
        for w in t:
            counts[w] = counts.get(w, 0) + 1
        for w, c in counts.items():
            rows.append(r)
            cols.append(idx[w])
            vals.append(c / len(t) * math.log((n + 1) / (df[w] + 1)))
    m = torch.zeros(n, len(vocab), dtype=torch.float64)
    if vals:
        m[torch.tensor(rows), torch.tensor(cols)] = torch.tensor(vals, dtype=torch.float64)
    return truncated_svd(m.to(dev), dims)


def truncated_svd(m, k: int):
    import torch

    u, s, _ = torch.linalg.svd(m, full_matrices=False)
    k = max(1, min(k, s.numel()))
    return (u[:, :k] * s[:k]).float()


def pca_reduce(x, dims: int):
    xc = x - x.mean(0, keepdim=True)
    return truncated_svd(xc.double(), dims)


def tsne_2d(x, iters: int = 1000, seed: int = 0, lr: float = 200.0):
    """Exact t-SNE (perplexity 30 capped at (n-1)/3, floor 2) on x's device."""
    import torch

    n = x.shape[0]
    dev = x.device
    perp = max(2.0, min(30.0, (n - 1) / 3.0))
    xx = x.double()
    sq = (xx * xx).sum(1)
    d = (sq[:, None] + sq[None, :] - 2.0 * xx @ xx.T).clamp_min(0.0)
    eye = torch.eye(n, dtype=torch.bool, device=dev)
    log_u = math.log(perp)
    beta = torch.ones(n, dtype=torch.float64, device=dev)
    lo = torch.zeros_like(beta)
    hi = torch.full_like(beta, float("inf"))
    # bisection on the per-row precision: entropy H(beta) falls as beta rises
    dmin = d.masked_fill(eye, float("inf")).min(1).values
    for _ in range(64):
        p = torch.exp(-(d - dmin[:, None]) * beta[:, None]).masked_fill(eye, 0.0)
        sp = p.sum(1).clamp_min(1e-300)
        h = torch.log(sp) + beta * ((d - dmin[:, None]) * p).sum(1) / sp
        up = h > log_u
        lo = torch.where(up, beta, lo)
        hi = torch.where(up, hi, beta)
        beta = torch.where(up, torch.where(torch.isinf(hi), beta * 2.0, (beta + hi) / 2.0),
                           (beta + lo) / 2.0)
    p = p / sp[:, None]
    p = ((p + p.T) / (2.0 * n)).clamp_min(1e-12).float()
    g = torch.Generator(device="cpu").manual_seed(seed)
    y = (torch.randn(n, 2, generator=g) * 1e-4).to(dev)
    iy = torch.zeros_like(y)
    gains = torch.ones_like(y)
    eye_f = eye
    for it in range(iters):
        exag = 4.0 if it < 100 else 1.0
        sy = (y * y).sum(1)
        num = (1.0 / (1.0 + sy[:, None] + sy[None, :] - 2.0 * y @ y.T)).masked_fill(eye_f, 0.0)
        q = (num / num.sum()).clamp_min(1e-12)
        w = (exag * p - q) * num
        dy = 4.0 * (w.sum(1, keepdim=True) * y - w @ y)
        mom = 0.5 if it < 250 else 0.8
        same = (dy > 0) == (iy > 0)
        gains = torch.where(same, gains * 0.8, gains + 0.2).clamp_min(0.01)
        iy = mom * iy - lr * gains * dy
        y = y + iy
        y = y - y.mean(0, keepdim=True)
    return y


def align(cur, ids: list[str], ref: dict | None):
    """Rotate/translate ``cur`` [n, 2] so points shared with the previous layout
    land where they were (orthogonal Procrustes, no scaling)."""
    import torch

    if not ref:
        return cur
    rows = [i for i, e in enumerate(ids) if e in ref]
    if len(rows) < 2:
        return cur
    a = cur[rows].double()
    b = torch.tensor([ref[ids[i]] for i in rows], dtype=torch.float64, device=cur.device)
    ca, cb = a.mean(0), b.mean(0)
    h = (a - ca).T @ (b - cb)
    u, _, vt = torch.linalg.svd(h)
    r = vt.T @ u.T
    return ((cur.double() - ca) @ r.T + cb).to(cur.dtype)


def normalize(c):
    m = c.abs().max()
    return c / m if float(m) > 0 else c


def project(inputs: list[Input], prev: dict | None = None, opts: Options | None = None,
            device=None) -> dict:
    """Returns {basis, model, total, unembedded, capped, points: [...]} with
    coordinates in [-1, 1]."""
    import numpy as np
    import torch

    opts = opts or Options()
    basis = choose_basis(inputs, opts.dense_threshold)
    used, unemb = select_inputs(inputs, basis)
    used, capped = apply_cap(used, opts.cap)
    res = {"basis": basis, "model": MODEL_TSNE, "total": len(used), "unembedded": unemb,
           "capped": capped, "points": []}
    if not used:
        return res
    dev = _device(device)
    if basis == BASIS_LEXICAL:
        red = tfidf_lsa([i.content for i in used], opts.lsa_dims, dev)
    else:
        x = torch.from_numpy(np.stack([np.asarray(i.embedding, dtype=np.float32).ravel()
                                       for i in used])).to(dev)
        red = pca_reduce(x, opts.pca_dims)
    if len(used) < opts.tiny_set:
        coords = red[:, :2] if red.shape[1] >= 2 else torch.cat(
            [red, torch.zeros(red.shape[0], 2 - red.shape[1], device=dev)], 1)
        res["model"] = MODEL_PCA
    else:
        coords = tsne_2d(red, opts.tsne_iters, opts.seed)
    ids = [i.entity_id for i in used]
    coords = normalize(align(coords.float(), ids, prev))
    for i, (x, y) in zip(used, coords.cpu().tolist()):
        res["points"].append({
            "id": i.entity_id, "x": x, "y": y, "tier": i.tier, "type": i.kind,
            "user": i.user, "userRef": i.user, "category": i.category,
            "confidence": i.confidence, "title": i.title,
            "preview": (i.content or "")[:opts.preview_chars],
            "observedAt": i.observed_at, "expiresAt": i.expires_at})
    return res


# ------------------------------------------------------------------ store side
def scope_key(workspace: str, user: str | None = None) -> str:
    return f"{workspace}|{user or ''}"


def gather_inputs(store, workspace: str, user: str | None = None, limit: int = 20000):
    """Latest active observation of every entity in scope, with its embedding."""
    from ..memory.model import META_CONSENT_CATEGORY, SCOPE_USER, SCOPE_WORKSPACE

    mems = store.list({SCOPE_WORKSPACE: workspace, **({SCOPE_USER: user} if user else {})},
                      limit=limit, strict=bool(user))
    emb = store.embedding_of([m.observation_id for m in mems])
    return [Input(m.id, m.content, emb.get(m.observation_id), m.tier, m.type,
                  m.scope.get(SCOPE_USER, ""), m.metadata.get(META_CONSENT_CATEGORY, ""),
                  m.confidence, m.title, m.observed_at, m.expires_at) for m in mems]


def fingerprint(inputs: list[Input]) -> str:
    """``count:max_observed_ns:embedded``; empty when there is nothing to lay out."""
    if not inputs:
        return ""
    mx = max(i.observed_at for i in inputs)
    emb = sum(1 for i in inputs if i.embedding is not None and len(i.embedding))
    return f"{len(inputs)}:{int(mx * 1e9)}:{emb}"


def _fp_count(fp: str) -> int:
    try:
        return int(fp.split(":")[0]) if fp else 0
    except ValueError:
        return 0


def _fp_eligible(fp: str) -> int:
    parts = (fp or "").split(":")
    try:
        return int(parts[2]) if len(parts) == 3 else 0
    except ValueError:
        return 0


def should_render(stored: dict | None, live: str, cfg: dict, now: float) -> bool:
    if stored is None:
        return True  # never rendered
    if stored.get("fingerprint") == live:
        return False  # unchanged: the layout is still valid
    eligibility_changed = _fp_eligible(live) != _fp_eligible(stored.get("fingerprint", ""))
    thr = int(cfg.get("changeThreshold") or 0)
    if not eligibility_changed and thr > 0 and \
            abs(_fp_count(live) - _fp_count(stored.get("fingerprint", ""))) < thr:
        return False  # not enough change yet
    if cfg.get("schedule"):
        if cron.next_fire(cfg["schedule"], float(stored.get("computed_at", 0.0))) >= now:
            return False  # rendered too recently
    return True


class ProjectionStore:
    """Rendered layouts in the memory store's ``memory_meta`` table, one row
    per scope key; every memory-api replica serves the same layout."""

    def __init__(self, store):
        self.s = store

    def load(self, key: str) -> dict | None:
        rows = self.s._q("SELECT value FROM memory_meta WHERE key = ?", ["projection:" + key])
        return json.loads(rows[0][0]) if rows else None

    def save(self, key: str, doc: dict):
        k = "projection:" + key
        with self.s._tx() as db:
            if db.execute("SELECT 1 FROM memory_meta WHERE key = ?", (k,)).fetchone():
                db.execute("UPDATE memory_meta SET value = ? WHERE key = ?", (json.dumps(doc), k))
            else:
                db.execute("INSERT INTO memory_meta (key, value) VALUES (?, ?)",
                           (k, json.dumps(doc)))


def render(store, workspace: str, user: str | None = None, opts: Options | None = None,
           device=None, now: float | None = None) -> dict:
    """Compute the scope's layout (aligned to the stored one) and store it."""
    ps = ProjectionStore(store)
    key = scope_key(workspace, user)
    inputs = gather_inputs(store, workspace, user)
    prev = ps.load(key)
    res = project(inputs, (prev or {}).get("coords"), opts, device)
    doc = {"fingerprint": fingerprint(inputs), "computed_at": now or time.time(),
           "basis": res["basis"], "model": res["model"], "total": res["total"],
           "unembedded": res["unembedded"], "capped": res["capped"],
           "coords": {p["id"]: [p["x"], p["y"]] for p in res["points"]}}
    ps.save(key, doc)
    return res


def from_stored(stored: dict, inputs: list[Input], preview_chars: int = 120) -> dict:
    """Serve the stored layout for the current rows (rows rendered since keep
    their coordinates; rows added after the render wait for the next one)."""
    pts = []
    for i in inputs:
        xy = stored.get("coords", {}).get(i.entity_id)
        if xy is None:
            continue
        pts.append({"id": i.entity_id, "x": xy[0], "y": xy[1], "tier": i.tier, "type": i.kind,
                    "user": i.user, "userRef": i.user, "category": i.category,
                    "confidence": i.confidence, "title": i.title,
                    "preview": (i.content or "")[:preview_chars], "observedAt": i.observed_at,
                    "expiresAt": i.expires_at})
    return {"basis": stored.get("basis", BASIS_UNKNOWN), "model": stored.get("model", ""),
            "total": len(pts), "unembedded": stored.get("unembedded", 0),
            "capped": stored.get("capped", False), "points": pts,
            "computedAt": stored.get("computed_at")}


class ProjectionWorker:
    """Renders each workspace whose policy has ``spec.projection.enabled`` when
    its fingerprint moved enough (``changeThreshold``) and the schedule allows;
    a workspace lease (shared with consolidation's lock store, trigger
    ``projection``) keeps replicas from rendering the same layout twice."""

    def __init__(self, store, policies, workspaces=None, interval_s: float = 300.0,
                 lock_store=None, opts: Options | None = None, device=None, now=time.time):
        from .consolidation import MetaLockStore

        self.store, self.policies, self.workspaces = store, policies, workspaces
        self.interval, self.opts, self.device, self.now = interval_s, opts, device, now
        self.locks = lock_store or MetaLockStore(store)
        self.ps = ProjectionStore(store)

    def _needs(self, ws, cfg) -> bool:
        live = fingerprint(gather_inputs(self.store, ws))
        if not live:
            return False  # no memories
        return should_render(self.ps.load(scope_key(ws)), live, cfg, self.now())

    def run_once(self) -> list[tuple[str, str]]:
        out = []
        pols = self.policies() if callable(self.policies) else self.policies
        for name, spec in pols:
            cfg = (spec or {}).get("projection") or {}
            if not cfg.get("enabled"):
                continue
            wss = self.workspaces(name) if self.workspaces else [name]
            for ws in wss:
                if not self._needs(ws, cfg):
                    out.append((ws, "skipped"))
                    continue
                ok, release = self.locks.try_lock(ws, "projection")
                if not ok:
                    out.append((ws, "lock_held"))
                    continue
                try:
                    if not self._needs(ws, cfg):  # a peer rendered it meanwhile
                        out.append((ws, "already_rendered"))
                        continue
                    t0 = self.now()
                    try:
                        res = render(self.store, ws, opts=self.opts, device=self.device,
                                     now=self.now())
                    except Exception as e:  # noqa: BLE001
                        RENDERS.labels(ws, name, "error", BASIS_UNKNOWN).inc()
                        log.error("projection render %s failed: %s", ws, e)
                        out.append((ws, "error"))
                        continue
                    RENDERS.labels(ws, name, "ok", res["basis"]).inc()
                    RENDER_SECONDS.labels(ws, name).observe(max(0.0, self.now() - t0))
                    out.append((ws, "rendered"))
                finally:
                    release()
        return out

    async def run(self):
        import asyncio

        _m.MEMORY_WORKER_RUNNING.labels("projection").set(1)
        try:
            while True:
                try:
                    await asyncio.to_thread(self.run_once)
                except Exception as e:  # noqa: BLE001
                    log.error("projection pass failed: %s", e)
                if self.interval <= 0:
                    return
                await asyncio.sleep(self.interval)
        finally:
            _m.MEMORY_WORKER_RUNNING.labels("projection").set(0)
