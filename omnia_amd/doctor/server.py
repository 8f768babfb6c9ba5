"""Doctor HTTP server (``internal/doctor/server.go`` semantics).

* ``GET /``                        -- a self-contained page that streams a run
* ``GET /api/v1/run?stream=true``  -- SSE: one ``data:`` frame per check result
  (``running`` markers included), then ``event: complete`` with the whole run
* ``POST /api/v1/run``             -- run synchronously, store it, ``{"runId"}``
* ``GET /api/v1/results/latest``   -- the last stored run (404 before any)
* ``GET /healthz``

``build`` returns a fresh :class:`Runner` per run, so the service URLs it probes
are re-resolved every time (a pod that moved is found again)."""
from __future__ import annotations

import json
import logging

from aiohttp import web

log = logging.getLogger("omnia.doctor")

INDEX = """<!doctype html><html><head><meta charset="utf-8"><title>omnia doctor</title>
<style>body{font:14px system-ui;margin:2em}td{padding:2px 10px}.pass{color:#080}
.fail{color:#b00}.skip{color:#888}.running{color:#06c}</style></head><body>
<h1>omnia doctor</h1><button id="go">Run checks</button> <span id="sum"></span>
<table id="t"></table><script>
const rows = {};
document.getElementById('go').onclick = () => {
  document.getElementById('t').innerHTML = ''; document.getElementById('sum').textContent = '';
  const es = new EventSource('api/v1/run?stream=true');
  es.onmessage = (e) => {
    const r = JSON.parse(e.data), k = r.category + '/' + r.name;
    let tr = rows[k];
    if (!tr) { tr = rows[k] = document.getElementById('t').insertRow(); }
    tr.innerHTML = '';
    for (const v of [r.category, r.name, r.status, r.detail || r.error || '',
                     r.duration_ms ? r.duration_ms.toFixed(0) + ' ms' : '']) {
      const td = tr.insertCell(); td.textContent = v; td.className = r.status; }
  };
  es.addEventListener('complete', (e) => {
    const s = JSON.parse(e.data).summary;
    document.getElementById('sum').textContent =
      `${s.passed} passed, ${s.failed} failed, ${s.skipped} skipped`;
    es.close();
  });
};
</script></body></html>"""


def build_app(build) -> web.Application:
    app = web.Application()
    state = {"latest": None}

    async def index(_):
        return web.Response(text=INDEX, content_type="text/html")

    async def run_sse(request):
        if request.query.get("stream") != "true":
            return web.Response(status=400, text="query parameter stream=true is required")
        resp = web.StreamResponse(headers={"Content-Type": "text/event-stream",
                                           "Cache-Control": "no-cache",
                                           "X-Accel-Buffering": "no"})
        await resp.prepare(request)
        try:
            runner = build()
        except Exception as e:  # noqa: BLE001
            log.exception("build runner failed")
            await resp.write(f"event: error\ndata: {json.dumps({'error': str(e)})}\n\n".encode())
            return resp

        async def emit(r):
            await resp.write(f"data: {json.dumps(r.to_json())}\n\n".encode())

        run = await runner.run(on_result=emit)
        state["latest"] = run
        await resp.write(f"event: complete\ndata: {json.dumps(run.to_json())}\n\n".encode())
        return resp

    async def run_trigger(_):
        try:
            runner = build()
        except Exception as e:  # noqa: BLE001
            return web.json_response({"error": str(e)}, status=500)
        run = await runner.run()
        state["latest"] = run
        return web.json_response({"runId": run.id})

    async def latest(_):
        if state["latest"] is None:
            return web.json_response({"error": "no run yet"}, status=404)
        return web.json_response(state["latest"].to_json())

    async def healthz(_):
        return web.json_response({"status": "ok"})

    app.router.add_get("/", index)
    app.router.add_get("/api/v1/run", run_sse)
    app.router.add_post("/api/v1/run", run_trigger)
    app.router.add_get("/api/v1/results/latest", latest)
    app.router.add_get("/healthz", healthz)
    return app
