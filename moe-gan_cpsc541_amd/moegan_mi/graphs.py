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
import torch

ACTIVE = None  # the SegmentedGraph being captured, if any


def eager(fn):
    """Run ``fn`` now; while a capture is active, also make it an eager segment of the replay."""
    if ACTIVE is None:
        return fn()
    return ACTIVE._eager(fn)


class SegmentedGraph:
    def __init__(self):
        self.items = []  # ("graph", CUDAGraph) | ("eager", fn)
        self.pool = None
        self._cur = None
        self.stream = None

    def capture(self, fn, *args, **kwargs):
        """Capture ``fn(*args, **kwargs)`` (which must already have run eagerly once with the same shapes,
        so every lazily sized buffer exists).  Returns fn's result (tensors in the graph pool)."""
        global ACTIVE
        assert ACTIVE is None, "nested capture"
        self.pool = torch.cuda.graph_pool_handle()
        self.stream = torch.cuda.Stream()
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
        self._end()
        r = fn()
        self.items.append(("eager", fn))
        self._begin()
        return r

    @property
    def n_graphs(self):
        return sum(1 for k, _ in self.items if k == "graph")

    def replay(self):
        for kind, x in self.items:
            if kind == "graph":
                x.replay()
            else:
                x()
