"""Host -> HBM batch prefetch for the training loop.

The reference moves each batch with a blocking ``.to(device)`` at the top of the step (t2i_moe_gan.py:1214-1216).
Here the DataLoader hands over pinned host tensors (``pin_memory=True``, train_model.py) and batch i+1 is copied
on a dedicated HIP stream while batch i trains; the compute stream waits on the copy's event only when it
reaches that batch, so the PCIe transfer overlaps the step instead of preceding it.  Tensors that arrive
unpinned are pinned first (a host-side copy).  On a non-HIP device the batches pass through unchanged.
"""
import torch


class DevicePrefetcher:
    def __init__(self, loader, device, dtype=torch.float32):
        self.loader = loader
        self.device = torch.device(device)
        self.dtype = dtype

    def __len__(self):
        return len(self.loader)

    @property
    def sampler(self):  # DistributedSampler.set_epoch stays reachable through the wrapper
        return getattr(self.loader, "sampler", None)

    def _issue(self, it, stream):
        try:
            batch = next(it)
        except StopIteration:
            return None
        with torch.cuda.stream(stream):
            out = []
            for t in batch:
                if torch.is_tensor(t) and t.device.type == "cpu":
                    if not t.is_pinned():
                        t = t.pin_memory()
                    t = t.to(self.device, non_blocking=True)
                    if t.is_floating_point() and t.dtype != self.dtype:
                        t = t.to(self.dtype)
                out.append(t)
            ev = torch.cuda.Event()
            ev.record(stream)
        return out, ev

    def __iter__(self):
        if self.device.type != "cuda":
            yield from self.loader
            return
        stream = torch.cuda.Stream(self.device)
        it = iter(self.loader)
        nxt = self._issue(it, stream)
        while nxt is not None:
            batch, ev = nxt
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            for t in batch:
                if torch.is_tensor(t) and t.is_cuda:
                    t.record_stream(cur)  # the copy stream's allocation is now used on the compute stream
            nxt = self._issue(it, stream)  # the next batch's copy overlaps this batch's step
            yield tuple(batch)
