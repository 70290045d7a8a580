"""MI355X-native vGPU device plugin for Kubernetes.

Imported as ``amdvgpu`` (see ``amdvgpu/__init__.py``): the project directory name is not a
valid Python identifier.

Subpackages
-----------
plugin    kubelet device-plugin (gRPC v1beta1) control plane: device backends (amdsmi /
          sysfs / fake), vGPU model, Allocate contract, topology-aware preferred
          allocation, legacy-preferred checkpoint controller, supervisor + CLI.
shim      Python side of the native data plane: locating/building the native libraries,
          ctypes bindings to the shared accounting region (libvgpu_region.so), and the
          container-runtime emulator that runs a process under an Allocate contract.
ops       ctypes bindings to the gfx950 calibration kernels (CU census, spin, copy).
models    ai-benchmark-equivalent workloads (ResNet-V2-50/152, VGG-16, DeepLab, LSTM) in
          stock PyTorch-ROCm, used by the benchmarks.
parallel  multi-GPU concerns: xGMI/PCIe topology scoring and the best-effort GPU-set
          policy used by GetPreferredAllocation.
utils     size parsing, logging.
"""
import os as _os

__version__ = "0.1.0"

PKG_DIR = _os.path.abspath(__path__[0])  # noqa: F821 (also correct when imported as amdvgpu)
REPO_DIR = _os.path.dirname(PKG_DIR)
LIB_DIR = _os.path.join(PKG_DIR, "lib")
NATIVE_DIR = _os.path.join(REPO_DIR, "native")
