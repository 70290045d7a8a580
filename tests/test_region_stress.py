"""Fault injection on the shared region (no GPU): concurrent charge/uncharge from many
processes against one quota, SIGKILL of processes mid-flight (possibly while holding the
robust mutex inside reclaim), then reclaim. The quota must never be exceeded and dead
processes' charges must be returned."""
import multiprocessing as mp
import os
import random
import signal
import time

import pytest

from amdvgpu.shim.region import Region

LIMIT = 1 << 30
CHUNK = 8 << 20


def _worker(path, seed, hold_event, stop_event, over_flag):
    r = Region(path)
    slot = r.register(os.getpid())
    rng = random.Random(seed)
    held = []
    while not stop_event.is_set():
        if held and (rng.random() < 0.45 or len(held) > 40):
            r.uncharge(slot, 0, held.pop())
        else:
            n = CHUNK * rng.randint(1, 4)
            if r.charge(slot, 0, n) == 0:
                held.append(n)
        if r.device(0)["used"] > LIMIT:
            over_flag.value = 1
        if rng.random() < 0.01:
            r.reclaim()
    hold_event.wait()
    # exit without unregistering: the region must reclaim us (like a crashed process)
    os._exit(0)


@pytest.mark.slow
def test_concurrent_quota_with_kills(region_path):
    r = Region(region_path, create=True)
    r.set_memory_limit(0, LIMIT)
    # spawn, not fork: the pytest process runs gRPC servers in other tests, and forking a
    # process with live gRPC threads can deadlock the child in gRPC's atfork handlers.
    ctx = mp.get_context("spawn")
    stop, hold = ctx.Event(), ctx.Event()
    over = ctx.Value("i", 0)
    procs = [ctx.Process(target=_worker, args=(region_path, i, hold, stop, over)) for i in range(12)]
    for p in procs:
        p.start()
    time.sleep(1.0)
    victims = procs[:4]
    for p in victims:
        os.kill(p.pid, signal.SIGKILL)
    time.sleep(1.0)
    stop.set()
    time.sleep(0.3)
    assert over.value == 0, "quota exceeded"
    assert r.device(0)["used"] <= LIMIT
    hold.set()
    for p in procs:
        p.join(timeout=30)
    # everybody is gone: reclaim returns every charge
    r.reclaim()
    assert r.device(0)["used"] == 0
    assert r.procs() == []
    r.close()
