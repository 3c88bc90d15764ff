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
# True while timing inside a HIP-graph capture: events become record nodes
EXTERNAL = False


@dataclasses.dataclass
class Rec:
    name: str
    bytes: int
    start: torch.cuda.Event
    end: torch.cuda.Event
    flops: int = 0
    mfma_s: float = 0.0  # ideal matrix-core time of the launch's instruction mix


class KernelTimer:
    """only: optional set of span names to time (others cost nothing).  Events
    come from a pool, created once per timer (event creation is a host API
    call; recording is a stream command)."""

    def __init__(self, only=None):
        self.recs: list[Rec] = []
        self.only = set(only) if only else None
        self._pool: list[torch.cuda.Event] = []

    def _event(self):
        if EXTERNAL:
            return torch.cuda.Event(enable_timing=True, external=True)
        return self._pool.pop() if self._pool else torch.cuda.Event(enable_timing=True)

    def reserve(self, n: int):
        """Pre-create n events (outside any timed region)."""
        for _ in range(n):
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()  # torch creates the HIP event lazily, at the first record
            self._pool.append(ev)

    def __enter__(self):
        global _active
        self._prev, _active = _active, self
        return self

    def __exit__(self, *exc):
        global _active
        _active = self._prev

    def summary(self):
        """{name: (launches, total_ms, total_bytes, total_flops, total_mfma_s)} —
        call after a synchronize."""
        out = {}
        for r in self.recs:
            n, ms, b, f, m = out.get(r.name, (0, 0.0, 0, 0, 0.0))
            out[r.name] = (n + 1, ms + r.start.elapsed_time(r.end), b + r.bytes, f + r.flops,
                           m + r.mfma_s)
        return out


def timing() -> bool:
    """Is a KernelTimer active (callers then split multi-launch calls into
    one timed span per launch)?"""
    return _active is not None


@contextlib.contextmanager
def span(name: str, nbytes: int, flops: int = 0, mfma_s: float = 0.0):
    t = _active
    """Times the launches inside; yields the record (None when no timer is
    active) so the caller can correct its counts once it knows which kernel
    ran (e.g. the fp32 64-row fallback's matrix time)."""
    if t is None or (t.only is not None and name not in t.only):
        yield None
        return
    s, e = t._event(), t._event()
    rec = Rec(name, int(nbytes), s, e, int(flops), float(mfma_s))
    s.record()
    yield rec
    e.record()
    t.recs.append(rec)
