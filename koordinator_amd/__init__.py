"""koordinator_amd — MI355X-native evaluator for koord-scheduler's per-pod Filter/Score pass.

The product is libkoordeval.so (koordinator_amd/csrc: C++ host state + gfx950 HIP kernels) behind the
C ABI in include/koord_eval.h.  This package holds its ctypes binding (abi, evaluator), the
Kubernetes-object helpers (model) and the synthetic cluster generator (synth).
"""
from . import abi, model  # noqa: F401
from .evaluator import Evaluator, KoordEvalError  # noqa: F401
