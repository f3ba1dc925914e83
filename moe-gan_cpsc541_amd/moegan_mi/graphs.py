"""Replay a whole training step as a chain of hipGraphs.

One C2 step enqueues ~900 kernels through ctypes; captured once, it replays with a
single graph launch per segment and no per-kernel host work.  The step code marks
the few places that must stay eager with ``eager(fn)``:
  * RCCL collectives (data-parallel gradient / expert-load all-reduces), which run
    between segments exactly as in the eager step;
  * launches that bench.py times with HIP events (the roofline kernel), so the events
    bracket that one kernel on the stream it runs on.
``eager(fn)`` called outside a capture simply runs ``fn`` -- the eager step is the
same code path.  All tensors the captured step allocates live in one private graph
memory pool, so addresses baked into the graphs stay valid for every replay.

Inputs are fixed buffers: refill them (``copy_`` / ``normal_``) before ``replay()``.
"""
import os
import weakref

import torch

ACTIVE = None  # the SegmentedGraph being captured, if any
_SIDES = weakref.WeakSet()  # live SideStreams: joined at every eager boundary (a segment must end joined)


def eager(fn):
    """Run ``fn`` now; while a capture is active, also make it an eager segment of the replay.  Every live side
    stream is joined first in both cases: an eager segment (an RCCL collective) may read what a side stream
    wrote, e.g. a block's expert weight gradients handed to a bucketed all-reduce (step.py)."""
    if ACTIVE is None:
        for side in list(_SIDES):
            side.join()
        return fn()
    return ACTIVE._eager(fn)


class SegmentedGraph:
    """``stream`` / ``pool``: share the capture stream (so the library's per-stream workspace) and the graph memory
    pool with other SegmentedGraphs that are replayed one at a time in stream order (the variants of one training
    loop): a pool's blocks that one capture freed are reused by the next capture, while tensors a graph still
    holds (its outputs) stay out of reach of the others."""

    def __init__(self, stream=None, pool=None):
        self.items = []  # ("graph", CUDAGraph) | ("eager", fn)
        self.pool = pool
        self._cur = None
        # capture stream (the library keeps one workspace per stream)
        self.stream = stream if stream is not None else torch.cuda.Stream()

    def run_eager(self, fn, *args, **kwargs):
        """Run ``fn`` eagerly on the capture stream: the warm-up that sizes every lazily allocated buffer,
        including the library's per-stream workspace, for the stream the capture will use."""
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            r = fn(*args, **kwargs)
        torch.cuda.current_stream().wait_stream(self.stream)
        return r

    def capture(self, fn, *args, **kwargs):
        """Capture ``fn(*args, **kwargs)`` (which must already have run once through ``run_eager`` with the
        same shapes, so every lazily sized buffer exists).  Returns fn's result (tensors in the graph pool)."""
        global ACTIVE
        assert ACTIVE is None, "nested capture"
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            ACTIVE = self
            try:
                self._begin()
                out = fn(*args, **kwargs)
                self._end()
            finally:
                ACTIVE = None
        torch.cuda.current_stream().wait_stream(self.stream)
        return out

    def _begin(self):
        g = torch.cuda.CUDAGraph()
        # thread-local: other threads (the process group's watchdog) keep making HIP calls meanwhile
        g.capture_begin(pool=self.pool, capture_error_mode="thread_local")
        self._cur = g

    def _end(self):
        self._cur.capture_end()
        self.items.append(("graph", self._cur))
        self._cur = None

    def _eager(self, fn):
        for side in list(_SIDES):
            side.join()
        self._end()
        r = fn()
        self.items.append(("eager", fn))
        self._begin()
        return r

    def release(self):
        """Drop the captured graphs and free the library's gradient-fold arena of the capture stream (the arena
        persists across replays; ops.fold_release)."""
        from . import ops
        self.items = []
        ops.fold_release(self.stream)

    @property
    def n_graphs(self):
        return sum(1 for k, _ in self.items if k == "graph")

    def replay(self):
        for kind, x in self.items:
            if kind == "graph":
                x.replay()
            else:
                x()


def side_streams_enabled(device):
    """Side streams only on request (MOEGAN_SIDE_STREAM=1): measured on the C2 step with hipGraph replay,
    overlapping the weight gradients with the data-gradient chain was slower (13.42 vs 13.02 ms/step)."""
    return torch.device(device).type == "cuda" and os.environ.get("MOEGAN_SIDE_STREAM", "0") == "1"


class SideStream:
    """Fork independent work (weight gradients) onto a second HIP stream and join it back.

    ``run(fn, *keep)`` makes the side stream wait for everything enqueued so far on the current
    stream, then enqueues ``fn`` on the side stream; ``keep`` are tensors allocated on the current
    stream that ``fn`` reads -- they are held until ``join()``, so the caching allocator cannot hand
    their memory to later current-stream work while the side stream may still read it.
    ``join()`` makes the current stream wait for the side stream.  Under capture the fork/join
    become graph edges (the side stream joins the capture through the event it waits on); a
    segment must be joined before it ends (``eager`` boundaries, the end of the step)."""

    def __init__(self, device, enabled=True):
        self.s = torch.cuda.Stream(device) if enabled else None
        self.keep = []
        self.pending = False
        _SIDES.add(self)

    def run(self, fn, *keep):
        if self.s is None:
            return fn()
        self.s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.s):
            r = fn()
        self.keep.extend(keep)
        self.pending = True
        return r

    def join(self):
        if self.pending:
            torch.cuda.current_stream().wait_stream(self.s)
            self.pending = False
            self.keep.clear()
