"""Agent-facing memory tools (``memory__remember`` / ``memory__recall`` /
``memory__open`` / ``memory__forget``), served in-process by the runtime's tool
executor against memory-api.  The reference gets these from its SDK and the
doctor probes ``memory__remember`` end to end (``internal/doctor/checks/memory.go:286``)."""
from __future__ import annotations

from ..tools.executor import InProcessHandler
from .model import SCOPE_AGENT, SCOPE_USER, SCOPE_WORKSPACE

CATEGORIES = ["memory:identity", "memory:preferences", "memory:health", "memory:location",
              "memory:context", "memory:history"]


def memory_tools(client, workspace: str = "", agent: str = "") -> InProcessHandler:
    def scope(ctx, agent_scoped=False):
        s = {SCOPE_WORKSPACE: workspace or getattr(ctx, "workspace", "")}
        if getattr(ctx, "user_id", ""):
            s[SCOPE_USER] = ctx.user_id
        if agent_scoped and agent:
            s[SCOPE_AGENT] = agent
        return s

    async def remember(args, ctx):
        s = scope(ctx)
        if SCOPE_USER not in s:
            return {"error": "no user identity on this session; nothing remembered"}
        about = args.get("about") if isinstance(args.get("about"), dict) else None
        meta = {"source_type": "user_requested"}
        if args.get("category"):
            meta["consent_category"] = args["category"]
        res = await client.save(s, args.get("content", ""), args.get("type") or "fact",
                                 float(args.get("confidence") or 0.8), meta, about)
        return {"id": res.get("memory", {}).get("id"), "action": res.get("action"),
                "potential_duplicates": res.get("potential_duplicates", [])}

    async def recall(args, ctx):
        s = scope(ctx)
        mems = await client.retrieve(s[SCOPE_WORKSPACE], s.get(SCOPE_USER, ""), agent,
                                     args.get("query", ""), int(args.get("limit") or 10))
        return {"memories": [{k: m.get(k) for k in ("id", "content", "type", "tier",
                                                    "confidence", "has_full_body")
                              if m.get(k) is not None} for m in mems]}

    async def open_(args, ctx):
        return await client.open(args.get("id", ""), scope(ctx)[SCOPE_WORKSPACE])

    async def forget(args, ctx):
        await client.forget(args.get("id", ""), scope(ctx)[SCOPE_WORKSPACE])
        return {"forgotten": args.get("id")}

    obj = {"type": "object"}
    fns = {
        "memory__remember": (
            "Store a durable fact about the user for future conversations.",
            {**obj, "properties": {"content": {"type": "string"},
                                   "category": {"type": "string", "enum": CATEGORIES},
                                   "type": {"type": "string"},
                                   "about": {"type": "object", "properties": {
                                       "kind": {"type": "string"}, "key": {"type": "string"}}}},
             "required": ["content"]}, remember),
        "memory__recall": (
            "Search remembered facts relevant to a query.",
            {**obj, "properties": {"query": {"type": "string"}, "limit": {"type": "integer"}},
             "required": ["query"]}, recall),
        "memory__open": ("Fetch the full body of one memory by id.",
                         {**obj, "properties": {"id": {"type": "string"}}, "required": ["id"]},
                         open_),
        "memory__forget": ("Forget one memory by id.",
                           {**obj, "properties": {"id": {"type": "string"}},
                            "required": ["id"]}, forget),
    }
    return InProcessHandler("omnia-memory", fns)
