"""Host half of the data path without a GPU: the background producer thread of
data/prefetch.StagedIterator (the reference's BackgroundGenerator)."""
import pytest


def test_background_producer_order_and_errors():
    """The host producer thread yields host(b) in order and re-raises its exceptions in the
    consumer (CPU only: no staging involved)."""
    from faster_distributed_training_amd.data.prefetch import _Producer
    p = _Producer(lambda b: b * b, 50, depth=2)
    assert [p.get() for _ in range(50)] == [b * b for b in range(50)]
    assert p.get() is _Producer._END
    p.close()

    def bad(b):
        if b == 3:
            raise ValueError("boom")
        return b
    p = _Producer(bad, 10)
    got = [p.get() for _ in range(3)]
    assert got == [0, 1, 2]
    with pytest.raises(ValueError):
        p.get()
    p.close()
    # abandoned early: close() stops the thread although the queue is full
    p = _Producer(lambda b: b, 1000, depth=1)
    p.get()
    p.close()
    assert not p.t.is_alive()

