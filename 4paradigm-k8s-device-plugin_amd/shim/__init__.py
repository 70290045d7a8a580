"""Python side of the native data plane (libvgpu_hip.so / libvgpu_region.so)."""
from .native import lib_path, shim_path, ensure_built  # noqa: F401
