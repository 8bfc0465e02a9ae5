"""optimobo_amd — MI355X-native hot path of OptiMOBO's acquisition maximisation.

GP posterior (Matern-5/2 ARD) → EHVI / HV-PoI / expected decomposition / EI → arg-max over a
large candidate batch, in hand-written gfx950 HIP kernels behind a ctypes C-ABI
(include/optimobo_hip.h).  Host modules mirror the reference's surface:
``optimobo_amd.problem``, ``optimobo_amd.scalarisations``, ``optimobo_amd.util_functions``,
``optimobo_amd.algorithms.optimisers``, ``optimobo_amd.result``.
"""
__version__ = "0.1.0"
