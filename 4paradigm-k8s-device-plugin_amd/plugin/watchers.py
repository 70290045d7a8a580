"""File-system and OS-signal watchers for the supervisor loop.

Reference: ``watchers.go`` — ``newFSWatcher`` (fsnotify on the device-plugin dir, :9-24)
and ``newOSWatcher`` (signal.Notify, :26-31). Here inotify is driven directly through
libc (ctypes; no extra dependency) with a stat-polling fallback, and signals are
funnelled into a queue that the supervisor selects on together with FS events.
"""
import ctypes
import ctypes.util
import os
import queue
import select
import signal
import struct
import threading

IN_CREATE = 0x100
IN_MOVED_TO = 0x80
IN_DELETE = 0x200
IN_NONBLOCK = 0o4000
IN_CLOEXEC = 0o2000000
_EVENT = struct.Struct("iIII")


class FSEvent:
    def __init__(self, name, op):
        self.name, self.op = name, op

    def __repr__(self):
        return f"FSEvent({self.name}, {self.op})"


class FSWatcher:
    """Posts FSEvent(path, "create"|"delete") for entries of ``directory`` into ``events``."""

    def __init__(self, directory, events, poll_interval=0.5, force_poll=False):
        self.dir = directory
        self.events = events
        self._stop = threading.Event()
        self._fd = -1
        libc_name = ctypes.util.find_library("c")
        self._libc = ctypes.CDLL(libc_name, use_errno=True) if libc_name else None
        if not force_poll and self._libc is not None and hasattr(self._libc, "inotify_init1"):
            fd = self._libc.inotify_init1(IN_NONBLOCK | IN_CLOEXEC)
            if fd >= 0 and self._libc.inotify_add_watch(fd, directory.encode(), IN_CREATE | IN_MOVED_TO | IN_DELETE) >= 0:
                self._fd = fd
            elif fd >= 0:
                os.close(fd)
        self._poll_interval = poll_interval
        self._thread = threading.Thread(target=self._run_inotify if self._fd >= 0 else self._run_poll,
                                        name="fswatcher", daemon=True)
        self._thread.start()

    @property
    def mode(self):
        return "inotify" if self._fd >= 0 else "poll"

    def _run_inotify(self):
        while not self._stop.is_set():
            r, _, _ = select.select([self._fd], [], [], 0.2)
            if not r:
                continue
            try:
                buf = os.read(self._fd, 4096)
            except BlockingIOError:
                continue
            except OSError:
                return
            off = 0
            while off + _EVENT.size <= len(buf):
                _wd, mask, _cookie, ln = _EVENT.unpack_from(buf, off)
                name = buf[off + _EVENT.size: off + _EVENT.size + ln].rstrip(b"\0").decode(errors="replace")
                off += _EVENT.size + ln
                op = "create" if mask & (IN_CREATE | IN_MOVED_TO) else "delete"
                self.events.put(FSEvent(os.path.join(self.dir, name), op))

    def _snapshot(self):
        out = {}
        try:
            for e in os.scandir(self.dir):
                try:
                    st = e.stat(follow_symlinks=False)
                    out[e.path] = (st.st_ino, st.st_ctime_ns)
                except OSError:
                    pass
        except OSError:
            pass
        return out

    def _run_poll(self):
        prev = self._snapshot()
        while not self._stop.wait(self._poll_interval):
            cur = self._snapshot()
            for p, key in cur.items():
                if prev.get(p) != key:
                    self.events.put(FSEvent(p, "create"))
            for p in prev:
                if p not in cur:
                    self.events.put(FSEvent(p, "delete"))
            prev = cur

    def close(self):
        self._stop.set()
        self._thread.join(timeout=2)
        if self._fd >= 0:
            os.close(self._fd)
            self._fd = -1


class OSWatcher:
    """Posts ("signal", signum) into ``events`` for the given signals (main thread only)."""

    def __init__(self, events, sigs=(signal.SIGHUP, signal.SIGINT, signal.SIGTERM, signal.SIGQUIT)):
        self.events = events
        self._old = {}
        for s in sigs:
            self._old[s] = signal.signal(s, self._handler)

    def _handler(self, signum, frame):
        self.events.put(("signal", signum))

    def close(self):
        for s, h in self._old.items():
            signal.signal(s, h)


def new_event_queue():
    return queue.Queue()
