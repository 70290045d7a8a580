"""Multi-GPU placement: xGMI/PCIe topology scoring and the best-effort GPU-set policy."""
from .topology import allocate_vdevices, best_effort, pair_score, set_score  # noqa: F401
