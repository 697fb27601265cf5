"""Forward renders of a stream of views with two in flight.

The reference renders evaluation views one after another (eval_lerf.py:320-350,
render_language_feature_map*; backend_renderer.py serves views on request).
One forward is a chain of short, latency-bound stages (preprocess, tile count,
scatter, sort, render); run back to back on one stream, each leaves the chip
partly idle.  `ViewStream` issues consecutive forwards on alternating HIP
streams, so view i+1's preprocess and binning run while view i renders, and
hands each result back one push later, made safe to use on the caller's
stream.  Values are those of the same forwards run one at a time (the same
kernels; only the issue order differs).

    vs = ViewStream()
    for cam in cams:
        prev = vs.push(lambda: rasterizer(...))    # the previous view's outputs (or None)
        ...
    rest = vs.flush()                              # the outputs still in flight

The inputs a render_fn reads (the model's tensors) must stay alive until the
outputs of that push have been handed back.
"""
from __future__ import annotations

from collections import deque

import torch


def _tensors(x):
    if isinstance(x, torch.Tensor):
        yield x
    elif isinstance(x, dict):
        for v in x.values():
            yield from _tensors(v)
    elif isinstance(x, (list, tuple)):
        for v in x:
            yield from _tensors(v)


class ViewStream:
    def __init__(self, device=None, depth: int = 2):
        if depth < 1:
            raise ValueError("ViewStream: depth must be >= 1")
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.device = dev
        # non-blocking streams: the caller's stream is often the legacy default
        # stream, with which torch's pool streams synchronise implicitly (an
        # event recorded there waits for every stream's earlier work, which
        # would serialise the views again)
        from ._lib import nonblocking_stream
        self.streams = [nonblocking_stream(dev) for _ in range(depth)]
        self.k = 0
        self.pending = deque()

    def push(self, render_fn):
        """Run render_fn (a no-grad forward returning tensors) on the next
        stream, behind everything enqueued on the caller's stream so far;
        returns the oldest result once `depth` are in flight, else None."""
        cur = torch.cuda.current_stream(self.device)
        s = self.streams[self.k % len(self.streams)]
        self.k += 1
        ready = torch.cuda.Event()
        ready.record(cur)
        s.wait_event(ready)
        with torch.cuda.stream(s), torch.no_grad():
            out = render_fn()
        done = torch.cuda.Event()
        done.record(s)
        self.pending.append((out, done))
        if len(self.pending) < len(self.streams):
            return None
        return self._take(cur)

    def flush(self) -> list:
        """The results still in flight, oldest first."""
        cur = torch.cuda.current_stream(self.device)
        out = []
        while self.pending:
            out.append(self._take(cur))
        return out

    def _take(self, cur):
        out, done = self.pending.popleft()
        cur.wait_event(done)
        for t in _tensors(out):
            t.record_stream(cur)   # allocated on a render stream, used on the caller's
        return out
