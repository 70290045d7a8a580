"""ctypes bindings to the hand-written gfx950 calibration kernels (libvgpu_kernels.so)."""
from .calib import cu_census, decode_location, scratch_hog, spin, spin_lds, stream_copy  # noqa: F401
