"""Per-kernel HIP-event timing used by bench.py (disabled by default: zero overhead).

``timed(name)`` brackets one C-ABI launch sequence with torch.cuda.Event records on torch's
current stream — the same stream the library launches on — so the elapsed time is that
sequence's device duration.
"""
import contextlib

import torch

_enabled = False
_events = {}


def enabled():
    return _enabled


def enable(on=True):
    global _enabled
    _enabled = on
    _events.clear()


@contextlib.contextmanager
def timed(name, nbytes=0):
    """nbytes = the launch's ALGORITHMIC HBM bytes (SURVEY.md §8d accounting), for the roofline."""
    if not _enabled:
        yield
        return
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    yield
    e.record()
    _events.setdefault(name, []).append((s, e, nbytes))


def summary():
    """{name: (launches, mean_ms, total_ms, total_bytes)} — call after torch.cuda.synchronize()."""
    out = {}
    for name, evs in _events.items():
        ms = [s.elapsed_time(e) for s, e, _ in evs]
        out[name] = (len(ms), sum(ms) / len(ms), sum(ms), sum(b for _, _, b in evs))
    return out
