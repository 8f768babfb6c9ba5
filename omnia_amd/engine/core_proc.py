"""Engine-core process: the GPU engine in its own OS process.

The serving process (asyncio runtime: gRPC/WebSocket turns, PromptPack
rendering, protobuf framing, session stores) and the engine loop (scheduler,
staging, hipGraph launches) used to share one interpreter.  Under load the
serving thread holds the GIL for tens of milliseconds at a time (GC passes,
bursts of 256 coroutine wake-ups), and every such hold delays the engine's next
launch while the GPU drains -- measured as 20-150 ms decode-step outliers on
the runtime turn path that the bare engine never shows.  Splitting them the way
the reference splits runtime and provider (the runtime reaches its LLM over the
network, ``internal/runtime`` -> PromptKit providers) removes the contention:

* the **core** (``python -m omnia_amd.engine.core_proc --fd N``) owns the GPU,
  runs :class:`LLMEngine` and, after every engine step, sends ONE frame with
  the step's tokens (detokenised, coalesced per request) and finishes;
* the **client** (:class:`EngineCoreClient`) is a drop-in for
  :class:`AsyncLLMEngine` (``generate`` / ``drop_session`` / ``has_session`` /
  ``tokenizer`` / ``shutdown``); a reader thread parses frames and hands each
  event loop its batch with one ``call_soon_threadsafe`` per frame.

Wire: a Unix socketpair, frames = little-endian u32 length + msgpack array.
  client -> core: ``[config, cfg]``, ``[add, rid, ids, params, sid]``,
  ``[abort, rid]``, ``[drop, sid]``, ``[call, qid, name, arg]``, ``[stop]``
  core -> client: ``[ready, info]``, ``[out, tokens, finishes]``,
  ``[reply, qid, value]``, ``[fatal, msg]``
  tokens = ``[[rid, text, last_token, n_tokens], ...]``;
  finishes = ``[[rid, reason, prompt_toks, output_toks, cached_toks, ttft], ...]``.

The client must be created before the serving process touches the GPU: the
core is started as a child process (never an exec of a GPU-initialised one).
"""
from __future__ import annotations

import asyncio
import collections
import dataclasses
import itertools
import logging
import os
import select
import socket
import struct
import subprocess
import sys
import threading
import time

import msgpack

from ..observability import timeline as TL

log = logging.getLogger("omnia.engine.core")

_HDR = struct.Struct("<I")


def _send(sock: socket.socket, obj, lock: threading.Lock | None = None) -> None:
    data = msgpack.packb(obj, use_bin_type=True)
    buf = _HDR.pack(len(data)) + data
    if lock is None:
        sock.sendall(buf)
    else:
        with lock:
            sock.sendall(buf)


class _Frames:
    """Incremental length-prefixed frame parser."""

    def __init__(self):
        self.buf = bytearray()

    def feed(self, data: bytes) -> list:
        self.buf += data
        out = []
        while len(self.buf) >= 4:
            (n,) = _HDR.unpack_from(self.buf)
            if len(self.buf) < 4 + n:
                break
            out.append(msgpack.unpackb(bytes(self.buf[4:4 + n]), raw=False,
                                       strict_map_key=False))
            del self.buf[:4 + n]
        return out


# ===================================================================== core side
class _Core:
    def __init__(self, sock: socket.socket, cfg_dict: dict):
        from .engine import EngineConfig, LLMEngine

        self.sock = sock
        dev = cfg_dict.pop("_device_index", None)
        if dev is not None and cfg_dict.get("device", "cuda") == "cuda":
            import torch

            torch.cuda.set_device(int(dev))
        if os.environ.get("OMNIA_ENGINE_SYNTHETIC", "0") == "1":
            from .synthetic import SyntheticEngine  # host-path capacity rehearsal

            self.eng = SyntheticEngine(EngineConfig(**cfg_dict))
        else:
            self.eng = LLMEngine(EngineConfig(**cfg_dict))
        self.reqs: dict = {}  # rid -> Sequence
        self.tok_out: dict = {}  # rid -> [parts, last_tok, n]
        self.fin_out: list = []
        self.frames = _Frames()
        self.stop = False
        self.faults: list = []
        self.fatal = False
        self._wlock = threading.Lock()

    # -- engine callbacks (engine thread == this thread)
    def _on_token(self, s, tok, text):
        e = self.tok_out.get(s.request_id)
        if e is None:
            self.tok_out[s.request_id] = [[text] if text else [], tok, 1 if tok is not None else 0]
        else:
            if text:
                e[0].append(text)
            if tok is not None:
                e[1] = tok
                e[2] += 1

    def _on_finish(self, s):
        self.reqs.pop(s.request_id, None)
        self.fin_out.append([s.request_id,
                             s.finish_reason.value if s.finish_reason else None,
                             len(s.prompt), len(s.output), s.prefix_hit, s.ttft()])

    # -- commands
    def _handle(self, m):
        op = m[0]
        eng = self.eng
        if op == "add":
            from .sampling_params import SamplingParams
            from ..utils.arrivals import mark

            mark("engine_add")

            _, rid, ids, params, sid = m
            try:
                s = eng.add_request(ids, SamplingParams(**params), sid, rid,
                                    on_token=self._on_token, on_finish=self._on_finish)
                self.reqs[rid] = s
            except Exception as e:  # noqa: BLE001 -- reported to the requester
                self.fin_out.append([rid, "error:" + str(e), len(ids), 0, 0, None])
        elif op == "abort":
            s = self.reqs.get(m[1])
            if s is not None and not s.is_finished:
                eng.abort(s.seq_id)
        elif op == "drop":
            eng.drop_session(m[1])
        elif op == "call":
            _, qid, name, arg = m
            try:
                val = self._call(name, arg)
            except Exception as e:  # noqa: BLE001
                val = {"error": str(e)}
            _send(self.sock, ["reply", qid, val], self._wlock)
        elif op == "stop":
            self.stop = True

    def _call(self, name, arg):
        eng = self.eng
        if name == "has_session":
            return bool(eng.blocks.has_session(arg))
        if name == "sync":
            if eng.device.type == "cuda":
                import torch

                torch.cuda.synchronize(eng.device)
            return True
        if name == "health":
            now = time.monotonic()
            recent = [t for t in self.faults if now - t < 60.0]
            storm = len(recent) >= int(os.environ.get("OMNIA_ENGINE_MAX_FAULTS", "3"))
            return {"healthy": not (self.fatal or storm), "faults": len(self.faults)}
        if name == "stats":
            return {"timing": dict(eng.timing), "counters": dict(eng.counters),
                    "runner": {k: v for k, v in eng.runner.stats.items()},
                    "kv_blocks": eng.blocks.num_blocks, "block_size": eng.cfg.block_size,
                    "use_graphs": eng.runner.use_graphs,
                    "gpu_busy_s": eng.busy_seconds()}
        if name == "reset_timing":
            for k in eng.timing:
                eng.timing[k] = 0.0
            eng.runner.stats["gil_wait_s"] = 0.0
            eng.busy_seconds(reset=True)
            return True
        raise ValueError(f"unknown call {name!r}")

    def _fail_all(self, e: Exception):
        from .sequence import FinishReason

        eng = self.eng
        for s in list(eng.seqs.values()):
            eng.scheduler.abort(s.seq_id)
            s.finish_reason = FinishReason.ERROR
            eng._finalize(s)

    def run(self):
        from ..utils.pyprof import maybe_start

        maybe_start("engine-core")
        from ..utils.proc_tune import tune_serving_process

        tune_serving_process()
        eng = self.eng
        mc = eng.model_cfg
        _send(self.sock, ["ready", {"model": mc.name, "vocab": mc.vocab_size,
                                    "kv_blocks": eng.blocks.num_blocks,
                                    "device": str(eng.device), "pid": os.getpid()}])
        # A reader thread drains the socket while this thread sits in GPU waits:
        # read only between steps, a burst of new requests (256 prompts at a
        # wave start) filled the socket buffer during a 100+ ms prefill step and
        # the runtime's send blocked its event loop until the step ended.
        inbox: collections.deque = collections.deque()
        wake = threading.Event()
        gone = threading.Event()

        def reader():
            try:
                while True:
                    data = self.sock.recv(1 << 20)
                    if not data:
                        break
                    msgs = self.frames.feed(data)
                    if msgs:
                        inbox.extend(msgs)
                        wake.set()
            except OSError:
                pass
            gone.set()
            wake.set()

        threaded = os.environ.get("OMNIA_CORE_INBOX_THREAD", "1") != "0"
        if threaded:
            threading.Thread(target=reader, name="omnia-core-inbox", daemon=True).start()
        else:
            self.sock.setblocking(False)
        fd = self.sock.fileno()
        while not self.stop:
            busy = eng.has_work()
            if threaded:
                if not busy and not inbox:
                    wake.wait(0.05)
                wake.clear()
            else:  # read only between steps (A/B switch)
                r, _, _ = select.select([fd], [], [], 0 if busy else 0.05)
                if r:
                    try:
                        data = self.sock.recv(1 << 20)
                    except BlockingIOError:
                        data = None
                    if data == b"":
                        gone.set()
                    elif data:
                        inbox.extend(self.frames.feed(data))
            while inbox:
                self._handle(inbox.popleft())
            if gone.is_set() and not inbox:
                break  # client went away
            if TL.ENABLED and not eng.has_work() and not getattr(eng, "inflight", None):
                # idle (a wave ended): resolve the step events and write the buffer
                # (the pod's SIGTERM at the end would skip atexit)
                if getattr(eng, "_tl", None):
                    eng.tl_flush()
                elif TL._events:
                    TL.flush()
            if eng.has_work():
                try:
                    eng.step()
                except Exception as e:  # noqa: BLE001
                    log.exception("engine step failed")
                    self.faults.append(time.monotonic())
                    try:
                        eng.recover(e)  # fail live seqs, drop resident KV, keep serving
                    except Exception:  # noqa: BLE001
                        log.exception("engine recovery failed")
                        self._fail_all(e)
                        self.fatal = True
            if self.tok_out or self.fin_out:
                toks = [[rid, "".join(e[0]), e[1], e[2]] for rid, e in self.tok_out.items()]
                fins, self.fin_out = self.fin_out, []
                self.tok_out = {}
                if fins:
                    from ..utils.arrivals import mark

                    for _ in fins:
                        mark("engine_finish")
                if not threaded:
                    self.sock.setblocking(True)
                _send(self.sock, ["out", toks, fins], self._wlock)
                if not threaded:
                    self.sock.setblocking(False)
        eng.shutdown()


def core_main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="omnia engine-core process")
    ap.add_argument("--fd", type=int, required=True)
    a = ap.parse_args(argv)
    logging.basicConfig(level=os.environ.get("OMNIA_LOG_LEVEL", "INFO"))
    sock = socket.socket(fileno=a.fd)
    frames = _Frames()
    cfg = None
    while cfg is None:
        data = sock.recv(1 << 20)
        if not data:
            return 1
        for m in frames.feed(data):
            if m[0] == "config":
                cfg = m[1]
    try:
        core = _Core(sock, cfg)
    except Exception as e:  # noqa: BLE001
        log.exception("engine init failed")
        _send(sock, ["fatal", f"{type(e).__name__}: {e}"])
        return 1
    core.frames = frames
    core.run()
    return 0


# ===================================================================== client side
class _Shim:
    """``client.engine`` stand-in exposing what callers read off LLMEngine."""

    def __init__(self, model_cfg, tokenizer):
        self.model_cfg = model_cfg
        self.tokenizer = tokenizer


class EngineCoreClient:
    """Drop-in for :class:`AsyncLLMEngine` backed by an engine-core process."""

    def __init__(self, cfg, device_index: int | None = None, env: dict | None = None,
                 start_timeout: float = 900.0):
        from ..models.config import resolve
        from .tokenizer import make_tokenizer

        self.cfg = cfg
        if cfg.checkpoint:
            from ..models.loader import config_from_hf

            mc = config_from_hf(cfg.checkpoint, cfg.model)
        else:
            mc = resolve(cfg.model)
        self.engine = _Shim(mc, make_tokenizer(mc, cfg.tokenizer))
        a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock = a
        e = dict(os.environ)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        e["PYTHONPATH"] = os.pathsep.join([root] + [x for x in e.get("PYTHONPATH", "").split(
            os.pathsep) if x])
        e.update(env or {})
        self.proc = subprocess.Popen(
            [sys.executable, "-m", "omnia_amd.engine.core_proc", "--fd", str(b.fileno())],
            pass_fds=[b.fileno()], env=e)
        b.close()
        self._wlock = threading.Lock()
        d = dataclasses.asdict(cfg)
        if device_index is not None:
            d["_device_index"] = int(device_index)
        _send(a, ["config", d], self._wlock)
        self.frames = _Frames()
        self.info = self._wait_ready(start_timeout)
        self._rid = itertools.count()
        self._chans: dict = {}  # rid -> (loop, _Chan)
        self._calls: dict = {}  # qid -> [threading.Event, value]
        self._qid = itertools.count()
        self._closed = False
        self.error: Exception | None = None
        self._reader = threading.Thread(target=self._read_loop, name="omnia-core-reader",
                                        daemon=True)
        self._reader.start()

    def _wait_ready(self, timeout):
        t_end = time.monotonic() + timeout
        while True:
            if self.proc.poll() is not None:
                raise RuntimeError(f"engine core exited during start-up (rc={self.proc.returncode})")
            r, _, _ = select.select([self.sock], [], [], 1.0)
            if r:
                data = self.sock.recv(1 << 20)
                if not data:
                    raise RuntimeError("engine core closed the channel during start-up")
                for m in self.frames.feed(data):
                    if m[0] == "ready":
                        return m[1]
                    if m[0] == "fatal":
                        raise RuntimeError(f"engine core failed to start: {m[1]}")
            if time.monotonic() > t_end:
                self.proc.kill()
                raise TimeoutError("engine core did not become ready")

    # -- reader thread
    def _read_loop(self):
        from .engine import GenEvent

        sock = self.sock
        while True:
            try:
                data = sock.recv(1 << 20)
            except OSError:
                data = b""
            if not data:
                break
            for m in self.frames.feed(data):
                op = m[0]
                if op == "out":
                    per_loop: dict = {}
                    for rid, text, tok, n in m[1]:
                        ent = self._chans.get(rid)
                        if ent is not None:
                            per_loop.setdefault(ent[0], []).append(
                                (ent[1], GenEvent(text=text, token=tok, n_tokens=n)))
                    for rid, reason, pt, ot, ct, ttft in m[2]:
                        ent = self._chans.pop(rid, None)
                        if ent is None:
                            continue
                        if reason and reason.startswith("error:"):
                            ev = RuntimeError(reason[6:])
                        else:
                            ev = GenEvent(finished=True, finish_reason=reason, prompt_tokens=pt,
                                          output_tokens=ot, cached_tokens=ct, ttft=ttft)
                        per_loop.setdefault(ent[0], []).append((ent[1], ev))
                    for loop, batch in per_loop.items():
                        try:
                            loop.call_soon_threadsafe(_deliver, batch)
                        except RuntimeError:
                            pass
                elif op == "reply":
                    c = self._calls.get(m[1])
                    if c is not None:
                        c[1] = m[2]
                        c[0].set()
        # channel closed: fail everything still waiting
        self.error = self.error or RuntimeError("engine core exited")
        for rid, (loop, ch) in list(self._chans.items()):
            try:
                loop.call_soon_threadsafe(_deliver, [(ch, self.error)])
            except RuntimeError:
                pass
        self._chans.clear()
        for c in self._calls.values():
            c[0].set()

    # -- API
    @property
    def tokenizer(self):
        return self.engine.tokenizer

    def call(self, name: str, arg=None, timeout: float = 600.0):
        qid = next(self._qid)
        c = [threading.Event(), None]
        self._calls[qid] = c
        _send(self.sock, ["call", qid, name, arg], self._wlock)
        if not c[0].wait(timeout):
            raise TimeoutError(f"engine core call {name} timed out")
        self._calls.pop(qid, None)
        if isinstance(c[1], dict) and "error" in c[1] and len(c[1]) == 1:
            raise RuntimeError(c[1]["error"])
        return c[1]

    async def generate(self, prompt, params=None, session_id: str | None = None,
                       request_id: str | None = None):
        from .engine import GenEvent, _Chan
        from .sampling_params import SamplingParams

        if self.error is not None:
            raise self.error
        if isinstance(prompt, str):
            prompt = self.tokenizer.encode(prompt, add_bos=True)
        params = (params or SamplingParams()).validate()
        loop = asyncio.get_running_loop()
        rid = request_id or f"r{next(self._rid)}"
        q = _Chan()
        self._chans[rid] = (loop, q)
        from ..utils.arrivals import mark

        mark("runtime_submit")
        _send(self.sock, ["add", rid, list(prompt), dataclasses.asdict(params), session_id],
              self._wlock)
        done = False
        try:
            while True:
                await q.event.wait()
                q.event.clear()
                items, q.items = q.items, []
                text, last_tok, n = [], None, 0
                for ev in items:
                    if isinstance(ev, Exception):
                        done = True
                        raise ev
                    if ev.finished:
                        if n:
                            yield GenEvent(text="".join(text), token=last_tok, n_tokens=n)
                        done = True
                        yield ev
                        return
                    text.append(ev.text)
                    if ev.token is not None:
                        last_tok = ev.token
                    n += ev.n_tokens
                if n or text:
                    yield GenEvent(text="".join(text), token=last_tok, n_tokens=n)
        finally:
            if not done:
                self._chans.pop(rid, None)
                try:
                    _send(self.sock, ["abort", rid], self._wlock)
                except OSError:
                    pass

    def drop_session(self, session_id: str):
        _send(self.sock, ["drop", session_id], self._wlock)

    def has_session(self, session_id: str) -> bool:
        return bool(self.call("has_session", session_id))

    def synchronize(self):
        self.call("sync")

    def stats(self) -> dict:
        return self.call("stats")

    def health(self, timeout: float | None = None) -> bool:
        """False when the core died, reports a fault storm, or cannot answer within
        ``OMNIA_CORE_HEALTH_TIMEOUT_S`` (a hung GPU step blocks its loop) -- the
        cross-process form of the in-process engine watchdog."""
        if self._closed or self.error is not None or self.proc.poll() is not None:
            return False
        t = float(os.environ.get("OMNIA_CORE_HEALTH_TIMEOUT_S", "30")) if timeout is None \
            else timeout
        try:
            return bool(self.call("health", timeout=t).get("healthy"))
        except Exception:  # noqa: BLE001 - timeout / broken pipe
            return False

    def shutdown(self, timeout: float = 30.0):
        if self._closed:
            return
        self._closed = True
        try:
            _send(self.sock, ["stop"], self._wlock)
        except OSError:
            pass
        try:
            self.proc.wait(timeout)
        except subprocess.TimeoutExpired:
            self.proc.kill()  # our own child, by PID
            self.proc.wait(10)
        try:
            self.sock.close()
        except OSError:
            pass


def _deliver(batch):
    for ch, ev in batch:
        ch.items.append(ev)
        ch.event.set()


if __name__ == "__main__":
    sys.exit(core_main())
