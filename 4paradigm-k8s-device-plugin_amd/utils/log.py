"""Logging setup for the control plane (``--verbose`` maps onto levels)."""
import logging
import sys

_FMT = "%(asctime)s %(levelname).1s %(name)s: %(message)s"


def get_logger(name="amdvgpu", verbose=0):
    log = logging.getLogger(name)
    if not log.handlers:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter(_FMT))
        log.addHandler(h)
        log.propagate = False
    log.setLevel(logging.DEBUG if verbose > 0 else logging.INFO)
    return log
