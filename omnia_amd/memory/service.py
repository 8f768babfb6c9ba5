"""Memory service layer: store + embedder + device-resident vector indexes.

Mirrors ``internal/memory/api/service.go`` responsibilities:

* save -> structured-key dedup in the store, then embedding-similarity dedup
  (>= 0.95 auto-supersede, >= 0.85 surfaced as potential duplicates,
  ``internal/memory/types.go:128-132``);
* embeddings computed inline when an embedder is configured, otherwise left to
  the re-embed worker (``reembed_worker.go:81-148``);
* hybrid retrieval: ANN over-fetch (fanout x 4) from the workspace index,
  fused with FTS via RRF in the store;
* semantic retrieval with a CEL deny-filter over metadata (fails closed);
* consent classification (EE): PII regex categories upgrade the caller's claim;
* events to Redis Streams ``omnia:memory-events:<workspace>``
  (``internal/memory/api/event_publisher.go:37,123-130``).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time

from ..observability import metrics as M
from ..utils.cel import DenyFilter
from . import retrieval as R
from .model import (AUTO_SUPERSEDE_SIMILARITY, DUPLICATE_CANDIDATE_LIMIT,
                    META_CONSENT_CATEGORY, SCOPE_AGENT, SCOPE_USER, SCOPE_WORKSPACE,
                    SURFACE_DUPLICATE_SIMILARITY, Memory, normalize_scope)
from .store import MemoryStore, MultiTierRequest, NotFound
from .vector_index import VectorIndex

log = logging.getLogger("omnia.memory")

# upgrade-only severity of consent categories (SERVICE.md "Consent classification")
_SEVERITY = {"memory:health": 3, "memory:identity": 2, "memory:location": 2}


class MemoryService:
    def __init__(self, store: MemoryStore | None = None, embedder=None, publisher=None,
                 enterprise: bool = False, device=None, classify_pii: bool = True):
        self.store = store or MemoryStore()
        self.embedder = embedder
        self.publisher = publisher  # async callable(stream, event dict)
        self.enterprise = enterprise
        self.classify_pii = classify_pii
        self.device = device
        self.indexes: dict[str, VectorIndex] = {}
        self.policy_ranker = None  # EE: retrieval.tier_ranker_from_policy
        self.policy_half_life = R.HalfLife()
        self.embed_model = getattr(embedder, "model", "") if embedder else ""
        self.vec_seq = 0  # last memory_vector_log row this replica's indexes applied
        self.cache = None  # optional CachedStore (Redis) for list / search reads
        if embedder is not None:
            if getattr(embedder, "dim", 0):
                self.store.ensure_embedding_dim(embedder.dim)
            self._warm_indexes()

    # ------------------------------------------------------------ indexes
    def _index(self, workspace: str) -> VectorIndex | None:
        if self.embedder is None or not getattr(self.embedder, "dim", 0):
            return None
        idx = self.indexes.get(workspace)
        if idx is None:
            idx = self.indexes[workspace] = VectorIndex(self.embedder.dim, device=self.device)
        return idx

    def _warm_indexes(self):
        self.vec_seq = self.store.max_vector_seq()
        by_ws: dict[str, list] = {}
        for oid, ws, vec in self.store.embeddings(model=self.embed_model or None):
            if vec is not None and len(vec) == getattr(self.embedder, "dim", -1):
                by_ws.setdefault(ws, []).append((oid, vec.tolist()))
        for ws, items in by_ws.items():
            idx = self._index(ws)
            if idx is not None:
                idx.upsert(items)

    def sync_vectors(self) -> int:
        """Apply the store's vector changes since the last sync to this replica's
        device indexes (another replica's writes, deletes, supersessions): the
        database is the source of truth, the GPU index a per-replica cache."""
        if self.embedder is None:
            return 0
        applied = 0
        while True:
            rows = self.store.vector_changes(self.vec_seq)
            if not rows:
                return applied
            last: dict[str, tuple] = {}  # obs_id -> (workspace, op) of its latest change
            for seq, oid, ws, op in rows:
                last[oid] = (ws, op)
                self.vec_seq = seq
            ups = [o for o, (_, op) in last.items() if op == "upsert"]
            vecs = self.store.embedding_of(ups)
            dim = getattr(self.embedder, "dim", -1)
            by_ws: dict[str, list] = {}
            for oid, (ws, op) in last.items():
                if op == "upsert" and oid in vecs and len(vecs[oid]) == dim:
                    by_ws.setdefault(ws, []).append((oid, vecs[oid].tolist()))
                else:
                    idx = self.indexes.get(ws)
                    if idx is not None:
                        idx.remove([oid])
            for ws, items in by_ws.items():
                idx = self._index(ws)
                if idx is not None:
                    idx.upsert(items)
            applied += len(last)

    async def _invalidate(self, scope_or_ws) -> None:
        """Writes bump the workspace's read-cache version (cache.py)."""
        if self.cache is not None:
            scope = scope_or_ws if isinstance(scope_or_ws, dict) else \
                {SCOPE_WORKSPACE: scope_or_ws}
            await self.cache.bump(scope)

    async def list_cached(self, scope: dict, types=None, limit: int = 50, offset: int = 0):
        if self.cache is None:
            return self.store.list(scope, types, limit, offset)
        return await self.cache.list(scope, types, limit, offset)

    async def search_cached(self, scope: dict, query: str, limit: int = 10):
        if self.cache is None:
            return self.store.search(scope, query, limit)
        return await self.cache.search(scope, query, limit)

    def _drop_vectors(self, obs_ids):
        for idx in self.indexes.values():
            idx.remove(obs_ids)

    async def _embed(self, texts: list[str]):
        if self.embedder is None:
            return None
        t0 = time.perf_counter()
        try:
            v = await self.embedder.embed(texts)
            M.MEMORY_EMBED_SECONDS.observe(time.perf_counter() - t0)
            return v
        except Exception as e:  # noqa: BLE001 - degrade to FTS-only
            M.MEMORY_EMBED_ERRORS.inc()
            log.warning("embedding failed: %s", e)
            return None

    async def _publish(self, workspace: str, ev: dict):
        if self.publisher is None:
            return
        try:
            await self.publisher(f"omnia:memory-events:{workspace}", ev)
        except Exception as e:  # noqa: BLE001
            log.debug("memory event publish failed: %s", e)

    # ------------------------------------------------------------ classification
    def classify(self, mem: Memory) -> str | None:
        """EE consent classification: regex PII categories upgrade the claim."""
        claimed = (mem.metadata or {}).get(META_CONSENT_CATEGORY)
        if not (self.enterprise and self.classify_pii):
            return claimed
        from ..ee.redaction import classify_categories

        best = claimed
        for cat in classify_categories(mem.content):
            if _SEVERITY.get(cat, 0) > _SEVERITY.get(best or "", 0):
                if best != cat:
                    M.MEMORY_CLASSIFY_OVERRIDES.labels(**{"from": best or "", "to": cat,
                                                          "source": "regex"}).inc()
                best = cat
        if best:
            M.MEMORY_CLASSIFY_CATEGORY.labels(category=best, source="regex").inc()
        return best

    async def classify_async(self, mem: Memory) -> str | None:
        """Rules, then (EE, when ``self.embedding_classifier`` is prewarmed) the
        embedding classifier for content the rules do not place
        (``ee/pkg/privacy/classify/embedding.go``)."""
        best = self.classify(mem)
        emb = getattr(self, "embedding_classifier", None)
        claimed = (mem.metadata or {}).get(META_CONSENT_CATEGORY)
        if not (self.enterprise and self.classify_pii) or emb is None or \
                emb.centroids is None or (best and best != claimed):
            return best
        try:
            cat, _ = await emb.classify(mem.content)
        except Exception as e:  # noqa: BLE001
            M.MEMORY_EMBED_ERRORS.inc()
            log.debug("embedding classification failed: %s", e)
            return best
        if cat and _SEVERITY.get(cat, 0) > _SEVERITY.get(best or "", 0):
            if best != cat:
                M.MEMORY_CLASSIFY_OVERRIDES.labels(**{"from": best or "", "to": cat,
                                                      "source": "embedding"}).inc()
            M.MEMORY_CLASSIFY_CATEGORY.labels(category=cat, source="embedding").inc()
            return cat
        return best

    # ------------------------------------------------------------ API
    async def save(self, mem: Memory, require_user: bool = True) -> dict:
        mem.scope = normalize_scope(mem.scope)
        ws = mem.scope.get(SCOPE_WORKSPACE, "")
        cat = await self.classify_async(mem)
        if cat:
            mem.metadata = {**(mem.metadata or {}), META_CONSENT_CATEGORY: cat}
            if self.store.is_revoked(ws, mem.scope.get(SCOPE_USER, ""), cat):
                raise PermissionError(f"consent for {cat} revoked")
        vec = None
        dups = []
        if self.embedder is not None and mem.content:
            vv = await self._embed([mem.content])
            vec = vv[0] if vv else None
        if vec is not None and not mem.id:
            idx = self._index(ws)
            near = idx.search([vec], DUPLICATE_CANDIDATE_LIMIT * 4)[0] if idx is not None else []
            near = self._same_scope(near, mem.scope)
            if near and near[0][1] >= AUTO_SUPERSEDE_SIMILARITY and not (
                    mem.metadata or {}).get("about_kind"):
                ent = self.store.entity_of_observations([near[0][0]]).get(near[0][0])
                if ent:
                    mem.id = ent
                    res = self.store.save(mem, require_user=require_user)
                    with self.store._tx() as db:
                        prev = [r[0] for r in db.execute(
                            "SELECT id FROM memory_observations WHERE entity_id = ? AND id != ? "
                            "AND superseded_by IS NULL", (ent, res["observation_id"])).fetchall()]
                        self.store._log_vectors(db, "delete", prev)
                        db.execute("UPDATE memory_observations SET superseded_by = ? WHERE "
                                   "entity_id = ? AND id != ? AND superseded_by IS NULL",
                                   (res["observation_id"], ent, res["observation_id"]))
                    res.update(action="auto_superseded", supersedes=[near[0][0]],
                               supersede_reason="high_similarity")
                    self._after_write(ws, res, vec, [near[0][0]])
                    await self._publish(ws, {"type": "memory.saved", "id": res["id"],
                                             "action": res["action"]})
                    await self._invalidate(mem.scope)
                    return res
            for oid, sim in near:
                if sim >= SURFACE_DUPLICATE_SIMILARITY and len(dups) < DUPLICATE_CANDIDATE_LIMIT:
                    m = self.store.get(self.store.entity_of_observations([oid]).get(oid, ""))
                    if m is not None:
                        dups.append({"id": m.id, "content": m.content, "similarity": sim})
        res = self.store.save(mem, require_user=require_user)
        self._after_write(ws, res, vec, res.get("supersedes") or [])
        if dups:
            res["potential_duplicates"] = dups
        await self._publish(ws, {"type": "memory.saved", "id": res["id"], "action": res["action"]})
        await self._invalidate(mem.scope)
        return res

    def _same_scope(self, near, scope):
        if not near:
            return near
        ents = self.store.entity_of_observations([o for o, _ in near])
        keep = []
        for oid, sim in near:
            m = self.store.get(ents.get(oid, ""))
            if m is not None and m.observation_id == oid and \
                    m.scope.get(SCOPE_USER) == scope.get(SCOPE_USER) and \
                    m.scope.get(SCOPE_AGENT) == scope.get(SCOPE_AGENT):
                keep.append((oid, sim))
        return keep

    def _after_write(self, ws, res, vec, superseded):
        if superseded:
            self._drop_vectors(superseded)
        if vec is not None:
            self.store.set_embedding(res["observation_id"], vec, self.embed_model)
            idx = self._index(ws)
            if idx is not None:
                idx.upsert([(res["observation_id"], vec)])

    async def update(self, entity_id: str, content=None, metadata=None, confidence=None,
                     workspace: str | None = None) -> Memory:
        cur = self.store.get(entity_id, workspace)
        if cur is None:
            raise NotFound(entity_id)
        m = self.store.update(entity_id, content, metadata, confidence)
        self._drop_vectors([cur.observation_id])
        if content is not None and self.embedder is not None:
            vv = await self._embed([m.content])
            if vv:
                self._after_write(m.scope[SCOPE_WORKSPACE], {"observation_id": m.observation_id},
                                  vv[0], [])
        await self._publish(m.scope[SCOPE_WORKSPACE], {"type": "memory.updated", "id": m.id})
        await self._invalidate(m.scope)
        return m

    async def forget(self, entity_id: str, workspace: str | None = None) -> bool:
        ok = self.store.forget(entity_id, workspace)
        if ok:
            self._drop_vectors(self.store.observation_ids_of([entity_id]))
            await self._publish(workspace or "", {"type": "memory.forgotten", "id": entity_id})
            await self._invalidate(workspace or "")
        return ok

    async def delete_all(self, scope: dict) -> int:
        n, obs = self.store.delete_all(scope)
        self._drop_vectors(obs)
        await self._publish(scope.get(SCOPE_WORKSPACE, ""), {"type": "memory.deleted_all",
                                                            "count": n})
        await self._invalidate(scope)
        return n

    async def batch_delete(self, scope: dict, limit: int) -> int:
        n, obs = self.store.batch_delete(scope, limit)
        self._drop_vectors(obs)
        await self._invalidate(scope)
        return n

    async def supersede(self, source_ids: list[str], mem: Memory) -> dict:
        res = self.store.supersede(source_ids, mem)
        self._drop_vectors(self.store.observation_ids_of(source_ids))
        vv = await self._embed([mem.content]) if self.embedder is not None else None
        self._after_write(mem.scope[SCOPE_WORKSPACE], res, vv[0] if vv else None, [])
        await self._invalidate(mem.scope)
        return res

    async def ann(self, workspace: str, query: str, k: int):
        if self.embedder is None or not query.strip():
            return []
        vv = await self._embed([query])
        if not vv:
            return []
        self.sync_vectors()  # other replicas' writes since the last query
        idx = self._index(workspace)
        if idx is None:
            return []
        return idx.search([vv[0]], k)[0]

    async def retrieve_multi_tier(self, req: MultiTierRequest) -> list[Memory]:
        t0 = time.perf_counter()
        ann = await self.ann(req.workspace_id, req.query, R.HYBRID_FANOUT * R.ANN_OVERFETCH)
        # drop ANN hits whose observation went inactive since indexing
        dead = self.store.inactive_observation_ids([o for o, _ in ann])
        ann = [(o, s) for o, s in ann if o not in dead]
        if ann:
            out = self.store.retrieve_multi_tier_hybrid(req, ann)
            mode = "hybrid"
        else:
            out = self.store.retrieve_multi_tier(req)
            mode = "fts"
        M.MEMORY_RETRIEVE_SECONDS.labels(mode=mode).observe(time.perf_counter() - t0)
        return out

    async def retrieve_semantic(self, workspace: str, query: str, deny_cel: str = "",
                                limit: int = 10) -> list[Memory]:
        deny = DenyFilter(deny_cel)  # malformed -> raises (fail closed, HTTP 500)
        req = MultiTierRequest(workspace_id=workspace, query=query, limit=limit * 4)
        # workspace-wide: every tier of the workspace
        ann = await self.ann(workspace, query, R.HYBRID_FANOUT * R.ANN_OVERFETCH)
        mems = self._workspace_hybrid(req, ann)
        return [m for m in mems if deny.allowed(m.metadata)][:limit]

    def _workspace_hybrid(self, req: MultiTierRequest, ann):
        st = self.store
        hits = st._fts_ids(req.query, 5000)
        where, args = "e.workspace_id = ?", [req.workspace_id]
        ids = list(dict.fromkeys(list(hits) + [o for o, _ in ann]))
        if not ids:
            return []
        rows = st._select_active(where + " AND o.id IN (%s)" % ",".join("?" * len(ids)),
                                 args + ids)
        by_obs = {r[10]: st._row_to_memory(r) for r in rows}
        fts_rank, cos_rank = {}, {}
        for oid in sorted(hits, key=lambda o: hits[o]):
            m = by_obs.get(oid)
            if m and m.id not in fts_rank:
                fts_rank[m.id] = len(fts_rank) + 1
        for oid, _ in ann:
            m = by_obs.get(oid)
            if m and m.id not in cos_rank:
                cos_rank[m.id] = len(cos_rank) + 1
        fused = R.rrf_ranks(fts_rank, cos_rank)
        by_ent = {m.id: m for m in by_obs.values()}
        out = []
        for eid, s in sorted(fused.items(), key=lambda kv: -kv[1]):
            m = by_ent[eid]
            m.score = s
            out.append(m)
        return out[: req.limit]

    async def reembed(self, batch: int = 64, workspace: str | None = None) -> int:
        """One pass of the re-embed worker: backfill missing / stale vectors."""
        if self.embedder is None:
            return 0
        rows = self.store.reembed_backlog(workspace, self.embed_model, batch)
        if not rows:
            return 0
        vecs = await self._embed([r[1] for r in rows])
        if not vecs:
            return 0
        for (oid, _content, ws), v in zip(rows, vecs):
            self._after_write(ws, {"observation_id": oid}, v, [])
        return len(rows)

    def stats(self, workspace: str) -> dict:
        s = self.store.stats(workspace, self.embed_model)
        M.MEMORY_EMBED_COVERAGE.labels(workspace=workspace).set(s["embedding_coverage"])
        M.MEMORY_REEMBED_BACKLOG.labels(workspace=workspace).set(s["reembed_backlog"])
        return s


def memory_to_event_json(m: Memory) -> str:
    return json.dumps(m.to_json())
