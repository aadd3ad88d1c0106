"""KubeOperator-AMD: MI355X-native Kubernetes cluster lifecycle manager with a bundled PyTorch-ROCm
training stack (gfx950 HIP kernels, RCCL data parallelism)."""
__version__ = "0.1.0"
