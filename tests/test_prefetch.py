"""Pinned H2D staging (data/prefetch.py over the native PinnedPrefetcher): copies run on the
prefetcher's own stream, fenced by events in both directions, and the loaders that use
it (AG-News text batches, streamed CIFAR) produce exactly the batches of their unstaged
paths."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_stager_roundtrip_on_copy_stream(cuda):
    from faster_distributed_training_amd.data.prefetch import PinnedStager
    from faster_distributed_training_amd.ops import _native
    st = PinnedStager(cuda, 1 << 16, 3)
    assert st.pf.copy_stream != _native.stream_ptr(cuda)  # a stream of its own
    a = np.arange(1000, dtype=np.int64)
    b = torch.randn(7, 9)
    s, (da, db) = st.stage([a, b])
    st.acquire(s)
    assert da.device == cuda and da.dtype == torch.int64 and db.shape == (7, 9)
    assert torch.equal(da.cpu(), torch.from_numpy(a)) and torch.equal(db.cpu(), b)
    st.release(s)
    with pytest.raises(ValueError):
        st.stage([np.zeros(1 << 17, dtype=np.uint8)])


def test_stager_fences_slot_reuse(cuda):
    """The compute stream is kept busy so the copy stream would run ahead: a copy into a
    slot must wait for the (delayed) readers of that slot's previous batch, and every
    reader must wait for its own copy."""
    from faster_distributed_training_amd.data.prefetch import PinnedStager
    st = PinnedStager(cuda, 1 << 20, 3)
    big = torch.randn(4096, 4096, device=cuda)
    n = 12
    sums = []
    for k in range(n):
        s, (d,) = st.stage([np.full(1 << 18, k + 1, dtype=np.float32)])
        for _ in range(3):
            big = big @ big * 1e-4  # delays the reader of slot s on the compute stream
        st.acquire(s)
        sums.append(d.sum())  # reads the slot after the delay
        st.release(s)
    got = torch.stack(sums).cpu()
    want = torch.tensor([(k + 1) * float(1 << 18) for k in range(n)])
    assert torch.equal(got, want), got


def test_text_loader_pinned_matches_unstaged(cuda):
    from faster_distributed_training_amd.data.agnews import TextBatchLoader, synthetic_agnews
    store = synthetic_agnews(600, seed=3)
    for resident in (True, False):
        ld = TextBatchLoader(store, 32, cuda, seed=1, length_buckets=(64, 128, 256), resident=resident)
        assert ld.stager is not None
        ref = TextBatchLoader(store, 32, "cpu", seed=1, length_buckets=(64, 128, 256))
        n = 0
        for got, want in zip(ld, ref):
            for g, w in zip(got, want):
                assert g.device.type == "cuda" and torch.equal(g.cpu(), w)
            n += 1
        assert n == len(ref) and ld.stager.staged == n


def test_cifar_streamed_matches_resident(cuda):
    from faster_distributed_training_amd.data.cifar import DeviceCIFARLoader, synthetic_cifar
    data, tg = synthetic_cifar(640, seed=4)
    res = DeviceCIFARLoader(data, tg, 64, cuda, train=False, shuffle=True, seed=2, out_dtype=torch.float32)
    stm = DeviceCIFARLoader(data, tg, 64, cuda, train=False, shuffle=True, seed=2, out_dtype=torch.float32,
                            resident=False)
    assert stm.stager is not None and not hasattr(stm, "images")
    n = 0
    for (xa, ya), (xb, yb) in zip(res, stm):
        assert torch.equal(xa, xb) and torch.equal(ya, yb)
        n += 1
    assert n == len(res) == stm.stager.staged
    # training augmentation: same per-rank RNG stream -> same crops / flips
    res = DeviceCIFARLoader(data, tg, 64, cuda, train=True, seed=2, out_dtype=torch.float32)
    stm = DeviceCIFARLoader(data, tg, 64, cuda, train=True, seed=2, out_dtype=torch.float32, resident=False)
    for (xa, ya), (xb, yb) in zip(res, stm):
        assert torch.equal(xa, xb) and torch.equal(ya, yb)


def test_submit_runs_on_worker_thread(cuda):
    """PinnedPrefetcher.submit: jobs issued by the native worker in order, wait() returns once
    a slot's job is issued, the device sees every batch."""
    from faster_distributed_training_amd.ops import _native
    nat = _native.native()
    pf = nat.PinnedPrefetcher(cuda.index or 0, 1 << 16, 3)
    dst = [torch.empty(1 << 14, dtype=torch.uint8, device=cuda) for _ in range(3)]
    srcs = [np.full(1 << 14, k, dtype=np.uint8) for k in range(9)]
    out = []
    for k in range(9):
        s = pf.submit([srcs[k].ctypes.data], [srcs[k].nbytes], [dst[k % 3].data_ptr()], 0)
        assert s == k % 3
        pf.wait(s, _native.stream_ptr(cuda))
        out.append(dst[s].float().mean())
    assert pf.submitted == 9
    pf.synchronize()
    assert [float(v) for v in torch.stack(out).cpu()] == [float(k) for k in range(9)]
