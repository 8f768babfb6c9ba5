"""Per-request state tracked by the scheduler."""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import Callable

from .sampling_params import SamplingParams

_ids = itertools.count()


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2


class FinishReason(str, enum.Enum):
    STOP = "stop"  # eos / stop token / stop string
    LENGTH = "length"  # max_tokens or context limit
    ABORT = "abort"
    ERROR = "error"


@dataclass(eq=False)  # identity semantics: `in` on lists must not compare token lists
class Sequence:
    prompt: list[int]
    params: SamplingParams
    session_id: str | None = None
    request_id: str = ""
    on_token: Callable | None = None  # callback(seq, new_token_id) on the engine thread
    on_finish: Callable | None = None  # callback(seq)
    seq_id: int = field(default_factory=lambda: next(_ids))
    output: list[int] = field(default_factory=list)
    blocks: list[int] = field(default_factory=list)
    num_cached: int = 0  # tokens whose KV is already in the cache
    status: SeqStatus = SeqStatus.WAITING
    finish_reason: FinishReason | None = None
    arrival: float = field(default_factory=time.perf_counter)
    first_token_time: float | None = None
    finish_time: float | None = None
    logprobs: list[float] = field(default_factory=list)
    preemptions: int = 0
    prefix_hit: int = 0
    pub_pages: int = 0  # leading prompt pages offered to the shared-prefix table
    pub_hash: bytes | None = None  # chain digest up to them
    text_tail: str = ""  # recent decoded text for stop-string matching
    slot: int = -1  # device token slot (ModelRunner.tok_slots), -1 = none
    slot_launch: int = -1  # launch that last used the slot
    n_real: int = 0  # output tokens whose value is known on the host
    guide: object = None  # K13 grammar matcher (engine/guided.py) for constrained output

    def __post_init__(self):
        self._plen = len(self.prompt)

    @property
    def all_tokens(self) -> list[int]:
        return self.prompt + self.output

    @property
    def length(self) -> int:
        return self._plen + len(self.output)

    @property
    def num_uncached(self) -> int:
        return self.length - self.num_cached

    @property
    def is_finished(self) -> bool:
        return self.status == SeqStatus.FINISHED

    def ttft(self) -> float | None:
        return None if self.first_token_time is None else self.first_token_time - self.arrival

    def latency(self) -> float | None:
        return None if self.finish_time is None else self.finish_time - self.arrival
