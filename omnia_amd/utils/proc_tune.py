"""Serving-process interpreter tuning (runtime / facade / engine-core).

A cyclic-GC pass holds the interpreter for its whole duration; on a serving
heap of thousands of coroutines, protobuf frames and token lists a full
collection takes tens of milliseconds, during which no turn starts, no frame
is relayed and (in the engine-core) no step is launched.  After start-up the
long-lived objects (modules, model config, compiled protobuf classes, the
tokenizer) are frozen out of collection, and the young-generation threshold
is raised so collections are rarer.

``OMNIA_GC_THRESHOLD`` = ``g0,g1,g2`` (default ``50000,20,100``); ``off``
keeps the interpreter defaults."""
from __future__ import annotations

import gc
import os


def tune_serving_process() -> None:
    spec = os.environ.get("OMNIA_GC_THRESHOLD", "50000,20,100")
    if spec == "off":
        return
    gc.collect()
    gc.freeze()
    gc.set_threshold(*[int(x) for x in spec.split(",")])
