"""Request / sequence state.

The reference has no generation loop at all: a "request" is one fan-out of the
same text to every worker and one raw pickled result back.
Here a :class:`Sequence` carries prompt ids, generated ids, sampling params and
per-token timestamps (TTFT / inter-token latency / end-to-end latency metrics).
"""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import List, Optional


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2
    ABORTED = 3


@dataclass
class SamplingParams:
    max_new_tokens: int = 64
    temperature: float = 0.0        # 0 -> greedy (argmax kernel)
    top_k: int = 0
    top_p: float = 1.0
    ignore_eos: bool = False
    seed: Optional[int] = None

    def to_dict(self):
        return dict(self.__dict__)

    @staticmethod
    def from_dict(d):
        return SamplingParams(**{k: v for k, v in (d or {}).items() if k in SamplingParams.__dataclass_fields__})


_ids = itertools.count(1)


@dataclass
class Sequence:
    prompt: List[int]
    params: SamplingParams = field(default_factory=SamplingParams)
    eos_token_id: Optional[int] = None
    seq_id: int = field(default_factory=lambda: next(_ids))
    request_id: Optional[str] = None
    output: List[int] = field(default_factory=list)
    status: SeqStatus = SeqStatus.WAITING
    num_cached: int = 0              # tokens whose K/V are in the paged cache
    chunk: int = 0                   # prefill tokens scheduled in the current step (0 = all the rest)
    slot: int = -1                   # pipeline microbatch slot
    arrival: float = field(default_factory=time.perf_counter)
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    token_times: List[float] = field(default_factory=list)
    finish_reason: Optional[str] = None

    def __post_init__(self):
        if not self.prompt:
            raise ValueError("empty prompt")
        self.prompt = [int(t) for t in self.prompt]

    @property
    def total_len(self) -> int:
        return len(self.prompt) + len(self.output)

    @property
    def prefill_len(self) -> int:
        """Tokens the current prefill step computes for this sequence (a chunk of a long prompt,
        or everything not yet in the KV cache)."""
        return self.chunk or (self.total_len - self.num_cached)

    def all_tokens(self) -> List[int]:
        return self.prompt + self.output

    def last_token(self) -> int:
        return self.output[-1] if self.output else self.prompt[-1]

    @property
    def finished(self) -> bool:
        return self.status in (SeqStatus.FINISHED, SeqStatus.ABORTED)

    def append(self, tok: int, now: Optional[float] = None) -> bool:
        """Append a generated token; returns True if the sequence just finished."""
        now = time.perf_counter() if now is None else now
        self.output.append(tok if type(tok) is int else int(tok))
        self.token_times.append(now)
        if self.first_token_time is None:
            self.first_token_time = now
        if (not self.params.ignore_eos and self.eos_token_id is not None and tok == self.eos_token_id):
            self.finish("eos", now)
        elif len(self.output) >= self.params.max_new_tokens:
            self.finish("length", now)
        return self.finished

    def finish(self, reason: str, now: Optional[float] = None):
        self.status = SeqStatus.FINISHED if reason != "abort" else SeqStatus.ABORTED
        self.finish_reason = reason
        self.finish_time = time.perf_counter() if now is None else now

    # metrics
    def ttft(self) -> Optional[float]:
        return None if self.first_token_time is None else self.first_token_time - self.arrival

    def latency(self) -> Optional[float]:
        return None if self.finish_time is None else self.finish_time - self.arrival

    def itl(self) -> List[float]:
        t = self.token_times
        return [b - a for a, b in zip(t, t[1:])]
