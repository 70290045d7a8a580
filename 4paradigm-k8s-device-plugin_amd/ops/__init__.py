"""ctypes bindings to the hand-written gfx950 calibration kernels (libvgpu_kernels.so)."""
from .calib import cu_census, spin, spin_lds, stream_copy, decode_location  # noqa: F401
