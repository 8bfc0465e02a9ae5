"""Scrambled Sobol' engine state for device-side candidate generation (omb_set_sobol).

The device generates point i of a scipy ``qmc.Sobol`` engine in closed form from the engine's
scrambled direction numbers and digital shift (see include/optimobo_hip.h, omb_set_sobol), so
this module only extracts that state: it is fixed by (d, seed, scramble) and costs one
engine construction on the host.  The sequence is the one the reference draws its MC cache
from (optimobo/algorithms/optimisers.py:121-141) and the one the host maximiser used before.
"""
import numpy as np
from scipy.stats import qmc


def engine_state(d, seed=None, scramble=True, bits=30):
    """(sv (d, bits) uint32, shift (d,) uint32, bits) of ``qmc.Sobol(d, scramble, seed, bits)``."""
    eng = qmc.Sobol(d=d, scramble=scramble, seed=seed, bits=bits)
    try:
        sv, shift, nbits = eng._sv, eng._shift, eng.bits
    except AttributeError as e:  # scipy's engine layout is private; fail loudly if it moved
        raise RuntimeError(f"scipy {__import__('scipy').__version__}: Sobol engine state not accessible ({e})")
    if nbits > 32:
        raise ValueError("device Sobol' generation supports bits <= 32")
    sv = np.ascontiguousarray(sv, dtype=np.uint32).reshape(d, nbits)
    shift = np.ascontiguousarray(shift, dtype=np.uint32).reshape(d)
    return sv, shift, int(nbits)
