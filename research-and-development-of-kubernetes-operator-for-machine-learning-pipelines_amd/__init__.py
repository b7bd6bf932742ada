"""mlopamd — MI355X-native MLflow model-deployment operator and serving runtime.

Control plane (``controller``): the reference's ``MlflowModel`` CRD, kopf-style
handlers, MLflow alias polling, SeldonDeployment emission, Prometheus-gated
canary with real rollback, HBM-aware placement.

Data plane (``runtime``, ``models``, ``ops``, ``parallel``): PyTorch-ROCm
serving runtime whose hot path is hand-written gfx950 HIP (MFMA) kernels,
continuous batching over a paged KV cache, hipGraph decode, TP/EP over RCCL.

The package directory carries the long repository name; ``mlopamd`` is its
import alias (a symlink at the repo root).
"""
__version__ = "0.1.0"
