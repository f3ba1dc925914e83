"""DevicePrefetcher (moegan_mi/prefetch.py), the build's replacement for the reference's blocking per-batch copy
(t2i_moe_gan.py:1262-1263): batch i+1 is copied host -> HBM on its own stream while batch i is consumed.

Checked on the GPU: batch order and values (pinned and unpinned host tensors, a ragged last batch), the dtype
cast, that the compute stream really waits for the copy (a long kernel queued ahead on the compute stream, then
the batch read on that stream), and that each batch's memory is recorded on the compute stream (its storage is
not handed to the next copy while the step that reads it may still run)."""
import pytest
import torch
from torch.utils.data import DataLoader, TensorDataset

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _loader(pin, n=10, bs=3, dtype=torch.float32):
    g = torch.Generator().manual_seed(3)
    imgs = (torch.rand(n, 3, 8, 8, generator=g) * 2 - 1).to(dtype)
    text = torch.randn(n, 16, generator=g).to(dtype)
    return DataLoader(TensorDataset(imgs, text), batch_size=bs, shuffle=False, pin_memory=pin), imgs, text


@pytest.mark.parametrize("pin", [True, False])
def test_prefetch_order_values(pin):
    from moegan_mi.prefetch import DevicePrefetcher
    dl, imgs, text = _loader(pin)
    pf = DevicePrefetcher(dl, DEV)
    assert len(pf) == len(dl) == 4
    seen = 0
    for i, (a, b) in enumerate(pf):
        assert a.is_cuda and b.is_cuda and a.dtype == torch.float32
        lo, hi = 3 * i, min(3 * i + 3, 10)
        assert torch.equal(a.cpu(), imgs[lo:hi]) and torch.equal(b.cpu(), text[lo:hi]), i
        seen += a.shape[0]
    assert seen == 10  # the ragged last batch (1 image) arrives too


def test_prefetch_casts_to_dtype():
    from moegan_mi.prefetch import DevicePrefetcher
    dl, imgs, _ = _loader(True, dtype=torch.float64)
    for i, (a, _) in enumerate(DevicePrefetcher(dl, DEV, dtype=torch.float32)):
        assert a.dtype == torch.float32
        assert torch.equal(a.cpu(), imgs[3 * i:3 * i + 3].float())


def test_prefetch_compute_stream_waits_and_records():
    from moegan_mi.prefetch import DevicePrefetcher
    dl, imgs, _ = _loader(True, n=12, bs=4)
    big = torch.randn(4096, 4096, device=DEV)
    recorded = []
    orig = torch.Tensor.record_stream

    def rec(self, stream):
        recorded.append((self.data_ptr(), stream))
        return orig(self, stream)
    torch.Tensor.record_stream = rec
    try:
        sums = []
        for a, _ in DevicePrefetcher(dl, DEV):
            for _ in range(4):  # keep the compute stream busy well past the next batch's copy
                big = torch.tanh(big @ big * 1e-3)
            sums.append(a.double().sum())  # enqueued on the compute stream after the copy's event
            cur = torch.cuda.current_stream()
            assert any(p == a.data_ptr() and s == cur for p, s in recorded), "batch not recorded on compute stream"
    finally:
        torch.Tensor.record_stream = orig
    torch.cuda.synchronize()
    for i, s in enumerate(sums):
        assert abs(float(s) - float(imgs[4 * i:4 * i + 4].double().sum())) < 1e-9, i
