"""ctypes binding of liboptimobo_hip.so (the C-ABI declared in include/optimobo_hip.h).

The shared library is built in-tree (``make -C optimobo_amd/csrc`` or
``python __graft_entry__.py``) and is REQUIRED: there is no CPU fallback.  Importing
this module on a machine without the library raises ImportError; calling into it without
a GPU fails with OMBError from ``omb_create``.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# OMB_LIB_PATH: another build of the same library (tests/test_asan_host.py loads the host-sanitized build of
# `make -C optimobo_amd/csrc asan` through it); the in-tree build otherwise
LIB_PATH = os.environ.get("OMB_LIB_PATH") or os.path.join(HERE, "liboptimobo_hip.so")

OMB_OK, OMB_EINVAL, OMB_EHIP, OMB_ENOMEM, OMB_ESTATE, OMB_EUNSUP, OMB_ENOTPD = 0, -1, -2, -3, -4, -5, -6
ERROR_NAMES = {OMB_EINVAL: "OMB_EINVAL", OMB_EHIP: "OMB_EHIP", OMB_ENOMEM: "OMB_ENOMEM",
               OMB_ESTATE: "OMB_ESTATE", OMB_EUNSUP: "OMB_EUNSUP", OMB_ENOTPD: "OMB_ENOTPD"}
KERNEL_MATERN52, KERNEL_RBF = 0, 1
EHVI_REFERENCE, EHVI_TEXTBOOK, EHVI_SIGMA = 0, 1, 2
EI_PLAIN, EI_PARETO, EI_CONSTRAINED = 0, 1, 2
EA_EI, EA_PARETO_EI = 0, 1
DEBUG_SPIN_LIMIT = 1
DEBUG_COV_TABLE = 2
DEBUG_FUSED_CHAIN = 3
DEBUG_ARGMAX_PASSES = 4
DEBUG_CHOL_MODE = 5
DEBUG_TIMING_STRIDE = 6
DEBUG_COV_FUSED = 8
DEBUG_SELECT_SEQ = 9
DEBUG_SYRK_GLDS = 10
MAX_OBJ, MAX_DIM, MAX_TRAIN, MAX_TRAIN_DENSE = 8, 256, 1024, 16384

_p = ctypes.c_void_p
_d = ctypes.c_double
_i = ctypes.c_int
_i64 = ctypes.c_int64
_dp = ctypes.POINTER(ctypes.c_double)

# name → (restype, argtypes); must match include/optimobo_hip.h exactly.
SIGNATURES = {
    "omb_abi_version": (_i, []),
    "omb_create": (_i, [_i, ctypes.POINTER(_p)]),
    "omb_destroy": (_i, [_p]),
    "omb_set_stream": (_i, [_p, _p]),
    "omb_use_own_stream": (_i, [_p]),
    "omb_synchronize": (_i, [_p]),
    "omb_last_error": (ctypes.c_char_p, [_p]),
    "omb_debug_set": (_i, [_p, _i, _i64]),
    "omb_set_gp": (_i, [_p, _i, _i, _i, _i, _p, _dp, _d, _p, _p]),
    "omb_kernel_block": (_i, [_p, _i, _p, _i64, _p]),
    "omb_posterior": (_i, [_p, _i, _p, _i64, _p, _p]),
    "omb_ehvi2d": (_i, [_p, _p, _p, _i64, _i64, _p, _i, _dp, _d, _d, _i, _p]),
    "omb_ehvi3d_mc": (_i, [_p, _p, _p, _i64, _i64, _p, _i, _dp, _d, _p, _p]),
    "omb_ehvi_mc": (_i, [_p, _i, _p, _p, _i64, _i64, _p, _i, _dp, _d, _p, _p]),
    "omb_ehvi_boxes": (_i, [_p, _i, _p, _p, _i64, _i64, _p, _i, _p, _i, _p]),
    "omb_hvpoi": (_i, [_p, _p, _p, _i64, _i64, _p, _i, _p]),
    "omb_expdec": (_i, [_p, _i, _p, _p, _i64, _i64, _p, _i, _i, _dp, _dp, _dp, _dp, _d, _p]),
    "omb_ei": (_i, [_p, _p, _p, _i64, _d, _d, _p]),
    "omb_ei_ext": (_i, [_p, _i, _i, _p, _p, _i64, _i64, _d, _d, _d, _p]),
    "omb_argmax_dev": (_i, [_p, _p, _i64, _i64, _p]),
    "omb_argmax": (_i, [_p, _p, _i64, _i64, _dp, ctypes.POINTER(_i64)]),
    # fused chain (host pointers for plan geometry)
    "omb_plan_ehvi2d": (_i, [_p, _p, _i, _dp, _d, _d, _i]),
    "omb_plan_ehvi3d_mc": (_i, [_p, _p, _i, _dp, _d]),
    "omb_plan_ehvi_mc": (_i, [_p, _i, _p, _i, _dp, _d]),
    "omb_plan_ehvi_boxes": (_i, [_p, _i, _p, _i, _p, _i]),
    "omb_plan_hvpoi": (_i, [_p, _p, _i]),
    "omb_plan_expdec": (_i, [_p, _i, _p, _i, _i, _dp, _dp, _dp, _dp, _d]),
    "omb_plan_ei": (_i, [_p, _d, _d]),
    "omb_plan_ei_ext": (_i, [_p, _i, _i, _d, _d, _d]),
    "omb_set_sobol": (_i, [_p, _i, _i, _p, _p, _dp, _dp]),
    "omb_sobol": (_i, [_p, _i64, _i64, _p]),
    "omb_eval": (_i, [_p, _p, _i64, _p]),
    "omb_eval_argmax": (_i, [_p, _p, _i64, _i64, _p]),
    "omb_eval_argmax_sobol": (_i, [_p, _i64, _i64, _p]),
    "omb_timing": (_i, [_p, _i]),
    "omb_timing_read": (_i, [_p, _dp, ctypes.POINTER(_i64)]),
    # Thompson sampling (TuRBO)
    "omb_posterior_cov": (_i, [_p, _i, _p, _i64, _p, _p]),
    "omb_cholesky": (_i, [_p, _p, _i64, _i64, _d, ctypes.POINTER(_i)]),
    "omb_posterior_samples": (_i, [_p, _i, _p, _i64, _p, _i, _d, _i, _p, _dp]),
    "omb_thompson_select": (_i, [_p, _p, _i, _i64, _p]),
    "omb_ea_search": (_i, [_p, _i, _d, _d, _p, _i, _i, _p, _p, _p, _p, _p, _p, _p]),
    # GP fit on the device
    "omb_gp_lml_grad": (_i, [_p, _i, _i, _i, _p, _p, _dp, _d, _d, _dp, _dp, _dp]),
    "omb_gp_lml_grad_batch": (_i, [_p, _i, _i, _i, _i, _p, _p, _dp, _dp, _d, _dp, _dp, _dp, _p]),
    "omb_gp_fit_state": (_i, [_p, _i, _i, _i, _i, _p, _p, _dp, _d, _d, _dp]),
}


class OMBError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


_LIB = None


def load():
    """Load and type the library once; raise ImportError if it has not been built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C optimobo_amd/csrc` "
                          "(or `python -c 'import __graft_entry__ as g; g.build()'`). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.omb_abi_version() != 1:
        raise ImportError("liboptimobo_hip.so ABI version mismatch")
    _LIB = lib
    return lib


def host_ptr(arr):
    """Pointer to a C-contiguous numpy array that the call reads synchronously (plan geometry)."""
    return ctypes.c_void_p(arr.ctypes.data)


def darr(values):
    """Host double array for the small by-value vectors of the ABI."""
    vals = [float(v) for v in values]
    return (ctypes.c_double * max(1, len(vals)))(*vals)
