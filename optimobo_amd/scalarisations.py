"""Scalarisation functions (optimobo/scalarisations.py:4-397), drop-in surface.

Same class names, constructor arguments, ``__call__(F, weights)``, ``set_bounds`` and output
shapes as the reference.  The host ``__call__`` evaluates on the few training points the
optimisers aggregate each iteration (optimisers.py:250, 443, 510); the per-candidate use
inside ``expected_decomposition`` runs on the GPU (omb_expdec) from ``device_spec()``.
"""
import numpy as np

# device ids — include/optimobo_hip.h OMB_SCAL_*
_IDS = {"WeightedSum": 0, "Tchebicheff": 1, "AugmentedTchebicheff": 2, "ModifiedTchebicheff": 3,
        "ExponentialWeightedCriterion": 4, "WeightedNorm": 5, "WeightedPower": 6, "WeightedProduct": 7,
        "PBI": 8, "IPBI": 9, "QPBI": 10, "APD": 11}


class Scalarisation:
    """Base: normalisation bounds, ``__call__`` → ``do`` → flattened ``_do`` (scalarisations.py:13-34)."""

    _param_names = ()

    def __init__(self, ideal_point=None, max_point=None):
        self.ideal_point = ideal_point
        self.max_point = max_point

    def __call__(self, *args, **kwargs):
        return self.do(*args, **kwargs)

    def do(self, F, weights, **args):
        return np.asarray(self._do(F, weights, **args)).flatten()

    def set_bounds(self, new_lower, new_upper):
        self.ideal_point = new_lower
        self.max_point = new_upper

    # -- shared pieces
    def _normalised(self, F):
        lo = np.asarray(self.ideal_point, dtype=np.float64)
        hi = np.asarray(self.max_point, dtype=np.float64)
        return (np.asarray(F, dtype=np.float64) - lo) / (hi - lo)

    @staticmethod
    def _rows(F):
        """View any input as (rows, k); the reference's 1-D branch equals the single-row case."""
        F = np.asarray(F, dtype=np.float64)
        return F if F.ndim == 2 else F.reshape(1, -1)

    def _do(self, F, weights):
        out = self._rowwise(self._normalised(self._rows(F)), np.asarray(weights, dtype=np.float64))
        return out if np.ndim(F) == 2 else out[0]

    # -- device
    def device_spec(self):
        """(scalarisation id, parameter list) for omb_expdec."""
        return _IDS[type(self).__name__], [float(getattr(self, p)) for p in self._param_names]


class WeightedSum(Scalarisation):
    def _rowwise(self, o, w):
        return (o * w).sum(axis=1)


class Tchebicheff(Scalarisation):
    def _rowwise(self, o, w):
        return (w * o).max(axis=1)


class AugmentedTchebicheff(Scalarisation):
    _param_names = ("alpha",)

    def __init__(self, ideal_point=None, max_point=None, alpha=0.0001):
        super().__init__(ideal_point, max_point)
        self.alpha = alpha

    def _rowwise(self, o, w):
        a = np.abs(o)
        return (a * w).max(axis=1) + self.alpha * a.sum(axis=1)


class ModifiedTchebicheff(Scalarisation):
    _param_names = ("alpha",)

    def __init__(self, ideal_point=None, max_point=None, alpha=1):
        super().__init__(ideal_point, max_point)
        self.alpha = alpha

    def _rowwise(self, o, w):
        a = np.abs(o)
        return ((a + (self.alpha * a.sum(axis=1))[:, None]) * w).max(axis=1)


class ExponentialWeightedCriterion(Scalarisation):
    _param_names = ("p",)

    def __init__(self, ideal_point=None, max_point=None, p=100, **kwargs):
        super().__init__(ideal_point, max_point)
        self.p = p

    def _rowwise(self, o, w):
        return (np.exp(self.p * w - 1) * np.exp(self.p * o)).sum(axis=1)


class WeightedNorm(Scalarisation):
    _param_names = ("p",)

    def __init__(self, ideal_point=None, max_point=None, p=3):
        super().__init__(ideal_point, max_point)
        self.p = p

    def _rowwise(self, o, w):
        return np.power((np.power(np.abs(o), self.p) * w).sum(axis=1), 1 / self.p)


class WeightedPower(Scalarisation):
    _param_names = ("p",)

    def __init__(self, ideal_point=None, max_point=None, p=3):
        super().__init__(ideal_point, max_point)
        self.p = p

    def _rowwise(self, o, w):
        return ((o ** self.p) * w).sum(axis=1)


class WeightedProduct(Scalarisation):
    def _rowwise(self, o, w):
        return ((o + 100000) ** w).prod(axis=1)


class _Penalty(Scalarisation):
    """PBI family: d1 = projection on w/‖w‖, d2 = distance to that line (scalarisations.py:261-268)."""

    _param_names = ("theta",)

    def __init__(self, ideal_point=None, max_point=None, theta=5):
        super().__init__(ideal_point, max_point)
        self.theta = theta

    @staticmethod
    def _d1_d2(o, w):
        u = w.reshape(1, -1) / np.linalg.norm(w)
        d1 = (o * u).sum(axis=1)
        d2 = np.linalg.norm(o - d1[:, None] * u, axis=1)
        return d1, d2

    def _do(self, F, weights):
        # PBI/IPBI/QPBI return a column (N, 1) for every input rank (flattened by do()).
        o = self._normalised(self._rows(F))
        return self._rowwise(o, np.asarray(weights, dtype=np.float64)).reshape(-1, 1)


class PBI(_Penalty):
    def _rowwise(self, o, w):
        d1, d2 = self._d1_d2(o, w)
        return d1 + self.theta * d2


class IPBI(_Penalty):
    def _rowwise(self, o, w):
        d1, d2 = self._d1_d2(o, w)
        return self.theta * d2 - d1


class QPBI(_Penalty):
    _param_names = ("theta", "alpha", "H")

    def __init__(self, ideal_point=None, max_point=None, theta=5, alpha=5.0, H=5.0):
        super().__init__(ideal_point, max_point, theta)
        self.alpha = alpha
        self.H = H

    def _rowwise(self, o, w):
        d1, d2 = self._d1_d2(o, w)
        k = o.shape[1]
        span = np.sum(np.asarray(self.max_point, np.float64) - np.asarray(self.ideal_point, np.float64))
        d_star = self.alpha * (np.reciprocal(float(self.H)) * np.reciprocal(float(k)) * span)
        return d1 + self.theta * d2 * (d2 / d_star)


class APD(Scalarisation):
    """Angle-penalised distance (RVEA), scalarisations.py:355-397."""

    _param_names = ("FE", "FE_max", "gamma")

    def __init__(self, ideal_point=None, max_point=None, FE=1, FE_max=10, gamma=0.010304664101210016):
        super().__init__(ideal_point, max_point)
        self.FE = FE
        self.FE_max = FE_max
        self.gamma = gamma

    def _do(self, f, w_vector):
        t = self._normalised(self._rows(f))
        length = np.linalg.norm(t, axis=1).reshape(-1, 1)
        w = np.asarray(w_vector, dtype=np.float64)
        if np.all(w == 0):
            w = np.full(t.shape[1], 1e-5)
        t = np.where(np.all(t == 0, axis=1, keepdims=True), 1e-5, t)
        cosang = (t / np.linalg.norm(t, axis=1, keepdims=True)) @ (w / np.linalg.norm(w))
        theta = np.arccos(np.clip(cosang, -1.0, 1.0)).reshape(-1, 1)
        return (1 + t.shape[1] * (self.FE / self.FE_max) * (theta / self.gamma)) * length


ALL = [WeightedSum, Tchebicheff, AugmentedTchebicheff, ModifiedTchebicheff, ExponentialWeightedCriterion,
       WeightedNorm, WeightedPower, WeightedProduct, PBI, IPBI, QPBI, APD]
