"""Reader of the node's GPU-time ledger files (``native/include/vgpu/ledger.h``) for the
monitor and tools: ``<board>/ledger.<gpu_id>``, written by the ``vgpu-ledger`` daemon the
plugin runs (``main.LedgerDaemon``). Layout version 1: a 128-byte header, then 1024
32-byte entries."""
import os
import struct
import time

MAGIC = 0x56474C31
VERSION = 1
HEADER = struct.Struct("<IIIiQQQqQ")   # magic version gpu_id n heartbeat samples period total_occ reads
ENTRY = struct.Struct("<iiQQQ")        # pid occ charged_ns busy_ns seen_ns
ENTRIES_AT = 128
MAX_PIDS = 1024


def monotonic_ns():
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC)


def read_ledger(path):
    """{gpu_id, heartbeat_ns, samples, period_ns, total_occ, reads, procs: [{pid, occ,
    charged_ns, busy_ns}]} or None when the file is not a ledger."""
    try:
        with open(path, "rb") as f:
            raw = f.read(ENTRIES_AT + ENTRY.size * MAX_PIDS)
    except OSError:
        return None
    if len(raw) < ENTRIES_AT:
        return None
    magic, version, gpu_id, n, hb, samples, period, total, reads = HEADER.unpack_from(raw, 0)
    if magic != MAGIC or version != VERSION:
        return None
    procs = []
    for i in range(max(0, min(n, MAX_PIDS))):
        off = ENTRIES_AT + i * ENTRY.size
        if off + ENTRY.size > len(raw):
            break
        pid, occ, charged, busy, _seen = ENTRY.unpack_from(raw, off)
        if pid > 0:
            procs.append({"pid": pid, "occ": occ, "charged_ns": charged, "busy_ns": busy})
    return {"gpu_id": gpu_id, "heartbeat_ns": hb, "samples": samples, "period_ns": period, "total_occ": total,
            "reads": reads, "procs": procs}


def read_board(board_dir):
    """Every ledger under ``board_dir``: {gpu_id: ledger}."""
    out = {}
    try:
        names = os.listdir(board_dir)
    except OSError:
        return out
    for fn in sorted(names):
        if fn.startswith("ledger.") and fn[7:].isdigit():
            led = read_ledger(os.path.join(board_dir, fn))
            if led:
                out[led["gpu_id"]] = led
    return out
