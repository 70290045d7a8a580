"""gfx950 calibration kernels (native/src/kernels/vgpu_kernels.hip) driven from PyTorch.

These are the measurement instruments of the data plane:

* :func:`cu_census` launches long-spinning single-wave workgroups that each record the
  (XCC, SE, SH, CU) they ran on, read from HW_REG_XCC_ID / HW_REG_HW_ID. The number of
  distinct CUs observed is the spatial partition a queue is actually confined to.
* :func:`spin` fixed-duration workgroups for duty-cycle measurements of the temporal
  limiter.
* :func:`stream_copy` 16 B/lane grid-stride copy: HBM bandwidth, or host-spill bandwidth
  when the source lives in spilled (host) memory.

The library is required: there is no PyTorch fallback, a missing build raises.
"""
import ctypes as C

from ..shim.native import KERNELS, lib_path

_lib = None


def _k():
    global _lib
    if _lib is None:
        L = C.CDLL(lib_path(KERNELS))
        L.vgpu_cu_census.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        L.vgpu_cu_census.restype = C.c_int
        L.vgpu_spin.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.vgpu_spin.restype = C.c_int
        L.vgpu_spin_lds.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.vgpu_spin_lds.restype = C.c_int
        L.vgpu_stream_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.vgpu_stream_copy.restype = C.c_int
        L.vgpu_scratch_hog.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        L.vgpu_scratch_hog.restype = C.c_int
        _lib = L
    return _lib


def decode_location(code):
    """(xcc, se, sh, cu) from a census code."""
    code = int(code)
    return (code >> 12) & 0xF, (code >> 8) & 0xF, (code >> 4) & 0xF, code & 0xF


def _stream(torch, device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def cu_census(nblocks=4096, spin_us=200, device=None):
    """Returns the set of distinct (xcc, se, sh, cu) tuples the workgroups ran on."""
    import torch
    device = torch.device(device or "cuda")
    out = torch.zeros(nblocks, dtype=torch.int32, device=device)
    rc = _k().vgpu_cu_census(C.c_void_p(out.data_ptr()), int(nblocks), int(spin_us), _stream(torch, device))
    if rc != 0:
        raise RuntimeError(f"vgpu_cu_census launch failed ({rc})")
    torch.cuda.synchronize(device)
    return {decode_location(c) for c in out.cpu().tolist()}


def spin(nblocks, spin_us, device=None, counter=None):
    """Launches ``nblocks`` workgroups spinning ``spin_us`` each (asynchronous)."""
    import torch
    device = torch.device(device or "cuda")
    ptr = C.c_void_p(counter.data_ptr()) if counter is not None else None
    rc = _k().vgpu_spin(int(nblocks), int(spin_us), ptr, _stream(torch, device))
    if rc != 0:
        raise RuntimeError(f"vgpu_spin launch failed ({rc})")


def spin_lds(nblocks, spin_us, lds_bytes, device=None):
    """Launches ``nblocks`` workgroups spinning ``spin_us`` each while holding
    ``lds_bytes`` of LDS (asynchronous): a grid dispatched over many rounds."""
    import torch
    device = torch.device(device or "cuda")
    rc = _k().vgpu_spin_lds(int(nblocks), int(spin_us), int(lds_bytes), _stream(torch, device))
    if rc != 0:
        raise RuntimeError(f"vgpu_spin_lds launch failed ({rc})")


def stream_copy(dst, src, nbytes=None):
    """Copies ``nbytes`` (default: all of src) from tensor src to tensor dst (asynchronous)."""
    import torch
    n = int(nbytes if nbytes is not None else src.numel() * src.element_size())
    if n > dst.numel() * dst.element_size() or n > src.numel() * src.element_size():
        raise ValueError("copy larger than a buffer")
    if n % 16:
        raise ValueError("stream_copy needs a multiple of 16 bytes")
    rc = _k().vgpu_stream_copy(C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()), n, _stream(torch, dst.device))
    if rc != 0:
        raise RuntimeError(f"vgpu_stream_copy launch failed ({rc})")


def scratch_hog(nblocks=4096, stride=2654435761 & 0x7FFFFFFF | 1, device=None):
    """Runs a kernel whose lanes each hold a 16 KiB private (scratch) array; returns the
    per-lane checksums. ROCr backs the private segment with a scratch allocation that
    never passes the allocation hooks (the shim accounts it from KFD's VRAM counter)."""
    import torch
    device = torch.device(device or "cuda")
    out = torch.empty(nblocks * 64, dtype=torch.int32, device=device)
    rc = _k().vgpu_scratch_hog(C.c_void_p(out.data_ptr()), int(nblocks), int(stride), _stream(torch, device))
    if rc != 0:
        raise RuntimeError(f"vgpu_scratch_hog launch failed ({rc})")
    return out
