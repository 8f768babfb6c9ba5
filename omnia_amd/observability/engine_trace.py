"""Engine-step observability (SURVEY §5.1 [design]).

Three optional views of the engine loop, all off by default and free when off:

* **OTel spans.** With tracing on (``observability/tracing.py``), every engine
  step exports an ``omnia.engine.prefill`` / ``omnia.engine.decode_step`` /
  ``omnia.engine.mixed_step`` span. Its interval is the host-side schedule +
  launch window (the device interval needs a sync; the untraced timeline has
  it). Attributes are ``omnia.engine.batch_size``, ``omnia.engine.tokens``,
  ``omnia.engine.kv_pages_used`` and ``omnia.engine.step``. The reference
  traces no engine (its provider is remote), so these extend its span set
  (``internal/tracing/tracing.go:214-296``) under the same ``omnia.`` prefix.
* **roctx markers** (``OMNIA_ROCTX=1``). Each engine step is a
  ``omnia.engine.step`` range, with a mark naming its kind and sizes. PyTorch-ROCm
  routes ``torch.cuda.nvtx`` to roctx, so ``rocprofv3 --marker-trace`` lines
  the ranges up with the kernels.
* **torch.profiler window** (``OMNIA_TORCH_PROFILE_DIR`` +
  ``OMNIA_TORCH_PROFILE_STEPS=a:b``). Steps a..b-1 are profiled (CPU + GPU
  activities), and a Chrome trace is written to the directory.
"""
from __future__ import annotations

import logging
import os
import time

from . import tracing

log = logging.getLogger("omnia.engine.trace")

SPAN_NAMES = {"prefill": "omnia.engine.prefill", "decode": "omnia.engine.decode_step",
              "mixed": "omnia.engine.mixed_step"}


def _nvtx():
    import torch

    return torch.cuda.nvtx


class EngineTrace:
    def __init__(self, device_type: str = "cuda", env=None):
        env = os.environ if env is None else env
        self.roctx = env.get("OMNIA_ROCTX", "0") == "1" and device_type == "cuda"
        self.prof_dir = env.get("OMNIA_TORCH_PROFILE_DIR", "")
        self.prof_window = None
        if self.prof_dir:
            a, _, b = env.get("OMNIA_TORCH_PROFILE_STEPS", "10:20").partition(":")
            self.prof_window = (int(a), int(b or int(a) + 10))
        self._prof = None
        self._open = False
        self.device_type = device_type
        self.spans = 0

    @property
    def active(self) -> bool:
        """Anything to do per step (checked before gathering step attributes)."""
        return self.roctx or tracing.tracer().enabled

    # -- one engine iteration
    def begin(self, step: int) -> None:
        if self.roctx:
            _nvtx().range_push("omnia.engine.step")
            self._open = True
        if self.prof_window is not None:
            self._profile_tick(step)

    def end(self) -> None:
        if self._open:
            _nvtx().range_pop()
            self._open = False

    def on_step(self, kind: str, ts: float, rows: int, ntok: int, kv_used: int,
                step: int) -> None:
        """A step was enqueued: ``ts`` = its schedule start (perf_counter)."""
        base = kind.replace("_sync", "")
        if self.roctx:
            _nvtx().mark(f"{SPAN_NAMES.get(base, base)} rows={rows} tokens={ntok}")
        if tracing.tracer().enabled:
            now_ns = time.time_ns()
            start_ns = now_ns - int((time.perf_counter() - ts) * 1e9)
            tracing.record_span(SPAN_NAMES.get(base, f"omnia.engine.{base}"), start_ns, now_ns, {
                "omnia.engine.batch_size": rows, "omnia.engine.tokens": ntok,
                "omnia.engine.kv_pages_used": kv_used, "omnia.engine.step": step,
                "omnia.engine.sync": kind.endswith("_sync")})
            self.spans += 1

    # -- torch.profiler window
    def _profile_tick(self, step: int) -> None:
        a, b = self.prof_window
        if self._prof is None and a <= step < b:
            import torch

            acts = [torch.profiler.ProfilerActivity.CPU]
            if self.device_type == "cuda":
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self._prof.__enter__()
        elif self._prof is not None and step >= b:
            self.stop_profile()

    def stop_profile(self) -> str | None:
        if self._prof is None:
            return None
        prof, self._prof = self._prof, None
        self.prof_window = None  # one window per process
        prof.__exit__(None, None, None)
        os.makedirs(self.prof_dir, exist_ok=True)
        path = os.path.join(self.prof_dir, f"engine_steps_{os.getpid()}.json")
        prof.export_chrome_trace(path)
        log.info("torch.profiler trace of the engine steps: %s", path)
        return path
