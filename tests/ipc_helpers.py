"""Helpers that spawned child processes import by name (torch.multiprocessing pickles
functions by reference, so they must live in an importable module)."""


def sum_consumer(q, out):
    """Receives a CUDA tensor through CUDA IPC and reports the sum of its elements (or the
    error that opening it raised, as a string)."""
    try:
        t = q.get(timeout=60)
        out.put(float(t.sum().item()))   # integer sum: exact
    except Exception as e:  # noqa: BLE001  (reported to the producer)
        out.put("consumer: " + repr(e)[:300])
