"""Byte-size parsing shared by the plugin and the tests.

Same grammar as the native shim's ``parse_size`` (native/src/core/config.cpp) and the
reference's ``get_limit_from_env`` [libvgpu.so multiprocess_memory_limit.c:101-111]:
``NNN[KkMmGgTt][iB|B]``; a bare number is bytes, ``m``/``M`` is MiB (the plugin emits
``"<MiB>m"``, reference ``server.go:488``).
"""
import re

_UNITS = {"": 1, "k": 1 << 10, "m": 1 << 20, "g": 1 << 30, "t": 1 << 40}
_RE = re.compile(r"^\s*(\d+)\s*([kKmMgGtT]?)(i?[bB])?\s*$")


def parse_size(text):
    """Returns bytes for ``text`` or raises ValueError."""
    m = _RE.match(str(text))
    if not m:
        raise ValueError(f"invalid size {text!r}")
    value = int(m.group(1)) * _UNITS[m.group(2).lower()]
    if value >= 1 << 64:
        raise ValueError(f"size {text!r} overflows 64 bits")
    return value


def format_mib(nbytes):
    """Formats bytes as the plugin's env value ``"<MiB>m"``."""
    return f"{int(nbytes) >> 20}m"
