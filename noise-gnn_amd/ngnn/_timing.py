"""Optional per-kernel device timing with HIP events (used by bench.py).

When a :class:`KernelTimer` is active, every libngnn launch made through
``ngnn.ops`` is bracketed by two events recorded on the stream the kernel is
launched on (torch's current stream, which is the stream handle passed to the
C ABI).  Each record carries the launch's ALGORITHMIC byte count (DESIGN.md
§Roofline) so achieved GB/s = bytes / event time.  Inactive: one ``is None``
check per launch.
"""
from __future__ import annotations

import contextlib
import dataclasses

import torch

_active = None


@dataclasses.dataclass
class Rec:
    name: str
    bytes: int
    start: torch.cuda.Event
    end: torch.cuda.Event
    flops: int = 0


class KernelTimer:
    def __init__(self):
        self.recs: list[Rec] = []

    def __enter__(self):
        global _active
        self._prev, _active = _active, self
        return self

    def __exit__(self, *exc):
        global _active
        _active = self._prev

    def summary(self):
        """{name: (launches, total_ms, total_bytes, total_flops)} — call after a synchronize."""
        out = {}
        for r in self.recs:
            n, ms, b, f = out.get(r.name, (0, 0.0, 0, 0))
            out[r.name] = (n + 1, ms + r.start.elapsed_time(r.end), b + r.bytes, f + r.flops)
        return out


@contextlib.contextmanager
def span(name: str, nbytes: int, flops: int = 0):
    t = _active
    if t is None:
        yield
        return
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    yield
    e.record()
    t.recs.append(Rec(name, int(nbytes), s, e, int(flops)))
