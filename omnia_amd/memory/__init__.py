"""memory-api: per-workspace agent memory (``cmd/memory-api``, ``internal/memory``).

Entities / observations / relations in SQLite (FTS5 with the porter stemmer in
place of Postgres ``tsvector``), vectors resident on the GPU and searched with
the hand-written K18 cosine top-k kernel in place of pgvector HNSW, embeddings
produced in-node (K17 mean-pool + L2) instead of by a remote provider.
Multi-tier ranking (confidence/frequency/recency 0.5/0.3/0.2) and hybrid FTS +
cosine RRF (k=60, fanout 100, ANN over-fetch x4) follow
``internal/memory/retrieve_multi_tier.go:126-129`` and
``retrieve_multi_tier_hybrid.go:37-41``.
"""
from .model import Memory, Tier, derive_tier  # noqa: F401
