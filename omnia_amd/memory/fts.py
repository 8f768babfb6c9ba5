"""Full-text query translation: Postgres ``websearch_to_tsquery('english', q)``
semantics onto SQLite FTS5 (porter stemmer).

``websearch_to_tsquery`` ANDs the terms, honours ``"quoted phrases"``, ``OR``
and ``-negation``, and drops English stopwords; the runtime's ambient recall
rewrites queries to OR semantics first (``internal/runtime/memory_retriever.go:430``).
"""
from __future__ import annotations

import re

STOPWORDS = frozenset("""a about above after again against all am an and any are as at be because
been before being below between both but by can did do does doing down during each few for from
further had has have having he her here hers herself him himself his how i if in into is it its
itself just me more most my myself no nor not now of off on once only or other our ours ourselves
out over own same she should so some such than that the their theirs them themselves then there
these they this those through to too under until up very was we were what when where which while
who whom why will with you your yours yourself yourselves remind""".split())

_TOKEN = re.compile(r'"[^"]*"|(?:(?<=\s)|^)-[^\s"]+|[^\s"]+', re.UNICODE)
_WORD = re.compile(r"[\w]+", re.UNICODE)


def _terms(text: str) -> list[str]:
    return [w.lower() for w in _WORD.findall(text) if w.lower() not in STOPWORDS]


def to_fts5(query: str) -> str:
    """Translate a websearch-style query into an FTS5 MATCH expression
    ('' when nothing meaningful remains)."""
    groups: list[list[str]] = [[]]  # OR of AND-groups
    negs: list[str] = []
    for tok in _TOKEN.findall(query or ""):
        if tok == "OR":
            if groups[-1]:
                groups.append([])
            continue
        if tok.startswith('"'):
            words = _WORD.findall(tok)
            if words:
                groups[-1].append('"' + " ".join(w.lower() for w in words) + '"')
            continue
        neg = tok.startswith("-") and len(tok) > 1  # "-word" at a word start negates
        ts = _terms(tok[1:] if neg else tok)
        if not ts:
            continue
        if neg:
            negs.extend(ts)
        else:
            groups[-1].extend(f'"{t}"' for t in ts)
    groups = [g for g in groups if g]
    if not groups:
        return ""
    expr = " OR ".join("(" + " AND ".join(g) + ")" if len(g) > 1 else g[0] for g in groups)
    if negs:
        expr = f"({expr}) NOT (" + " OR ".join(f'"{t}"' for t in negs) + ")"
    return expr


def to_or_query(query: str) -> str:
    """``toFTSOrQuery``: "alpha beta" -> "alpha OR beta" (ambient recall)."""
    f = (query or "").split()
    return query if len(f) <= 1 else " OR ".join(f)
