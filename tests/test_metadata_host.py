"""Host logic of the metadata build that needs no GPU: the batched count reads of a replay (metadata._Deferred)."""
import torch

from sparseconvnet import metadata as md


def test_deferred_reads_batch_and_order():
    """Queued reads are applied in queue order from one copy per round; work queued with then() runs once every
    read queued before it is applied; reads queued by that work make another round; _later reads at once when no
    replay is in progress."""
    d = md._Deferred(None)
    log = []
    d.read(torch.tensor([3, 4], dtype=torch.int64), lambda v: log.append(("a", v)))
    d.then(lambda: (log.append(("then", None)),
                    d.read(torch.tensor([7], dtype=torch.int64), lambda v: log.append(("c", v)))))
    d.read(torch.tensor([5], dtype=torch.int64), lambda v: log.append(("b", v)))
    assert log == []
    d.flush()
    assert log == [("a", [3, 4]), ("b", [5]), ("then", None), ("c", [7])]
    assert not d.reads and not d.after
    got = []
    md._later(torch.tensor([9, 8], dtype=torch.int64), got.extend)
    assert got == [9, 8]


def test_deferred_is_per_thread():
    """The replay in progress is thread-local: a prefetch on a worker thread does not defer the reads of another
    thread's build."""
    import threading
    md._TLS.defer = md._Deferred(None)
    try:
        seen = []
        th = threading.Thread(target=lambda: seen.append(md._defer()))
        th.start()
        th.join()
        assert seen == [None] and md._defer() is not None
    finally:
        md._TLS.defer = None
