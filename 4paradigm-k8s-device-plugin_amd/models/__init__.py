"""ai-benchmark-equivalent workloads in stock PyTorch-ROCm (random init, synthetic data)."""
from .aibench import CASES, Case, build_case, get_case  # noqa: F401
