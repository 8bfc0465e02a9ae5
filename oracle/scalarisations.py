"""Oracle: the twelve OptiMOBO scalarisations, batched over leading axes (fp64 numpy).

TEST INFRASTRUCTURE ONLY — see oracle/__init__.py.

Restates optimobo/scalarisations.py:4-397.  ``batched(F, w)`` maps F (..., k) → (...),
equal to the reference ``Scalarisation.__call__`` on a 2-D (M, k) array
(scalarisations.py:17-27, which flattens ``_do``'s result).  The ``ID`` values match the
device kernel's scalarisation switch (include/optimobo_hip.h, OMB_SCAL_*).
"""
import numpy as np


class _Base:
    ID = -1

    def __init__(self, ideal_point=None, max_point=None):
        self.ideal_point = ideal_point
        self.max_point = max_point

    def set_bounds(self, lo, hi):          # scalarisations.py:29-34
        self.ideal_point, self.max_point = lo, hi

    def norm(self, F):                      # (F − ideal)/(max − ideal), e.g. scalarisations.py:45
        lo = np.asarray(self.ideal_point, np.float64)
        hi = np.asarray(self.max_point, np.float64)
        return (np.asarray(F, np.float64) - lo) / (hi - lo)

    def __call__(self, F, weights):
        F = np.asarray(F, np.float64)
        return np.asarray(self.batched(F if F.ndim > 1 else F[None, :], np.asarray(weights, np.float64))).reshape(-1)

    def params(self):
        return []


class WeightedSum(_Base):                   # scalarisations.py:37-50
    ID = 0

    def batched(self, F, w):
        return np.sum(self.norm(F) * w, axis=-1)


class Tchebicheff(_Base):                   # scalarisations.py:53-72
    ID = 1

    def batched(self, F, w):
        return np.max(w * self.norm(F), axis=-1)


class AugmentedTchebicheff(_Base):          # scalarisations.py:76-109
    ID = 2

    def __init__(self, ideal_point=None, max_point=None, alpha=0.0001):
        super().__init__(ideal_point, max_point)
        self.alpha = alpha

    def batched(self, F, w):
        a = np.abs(self.norm(F))
        return np.max(a * w, axis=-1) + self.alpha * np.sum(a, axis=-1)

    def params(self):
        return [self.alpha]


class ModifiedTchebicheff(_Base):           # scalarisations.py:113-149
    ID = 3

    def __init__(self, ideal_point=None, max_point=None, alpha=1):
        super().__init__(ideal_point, max_point)
        self.alpha = alpha

    def batched(self, F, w):
        a = np.abs(self.norm(F))
        right = self.alpha * np.sum(a, axis=-1)
        return np.max((a + right[..., None]) * w, axis=-1)

    def params(self):
        return [self.alpha]


class ExponentialWeightedCriterion(_Base):  # scalarisations.py:153-173
    ID = 4

    def __init__(self, ideal_point=None, max_point=None, p=100, **kwargs):
        super().__init__(ideal_point, max_point)
        self.p = p

    def batched(self, F, w):
        return np.sum(np.exp(self.p * w - 1) * np.exp(self.p * self.norm(F)), axis=-1)

    def params(self):
        return [self.p]


class WeightedNorm(_Base):                  # scalarisations.py:177-197
    ID = 5

    def __init__(self, ideal_point=None, max_point=None, p=3):
        super().__init__(ideal_point, max_point)
        self.p = p

    def batched(self, F, w):
        return np.power(np.sum(np.power(np.abs(self.norm(F)), self.p) * w, axis=-1), 1 / self.p)

    def params(self):
        return [self.p]


class WeightedPower(_Base):                 # scalarisations.py:201-219
    ID = 6

    def __init__(self, ideal_point=None, max_point=None, p=3):
        super().__init__(ideal_point, max_point)
        self.p = p

    def batched(self, F, w):
        return np.sum((self.norm(F) ** self.p) * w, axis=-1)

    def params(self):
        return [self.p]


class WeightedProduct(_Base):               # scalarisations.py:222-238
    ID = 7

    def batched(self, F, w):
        return np.prod((self.norm(F) + 100000) ** w, axis=-1)


def _pbi_parts(objs, w):
    W = w / np.linalg.norm(w)               # scalarisations.py:261-263
    d1 = np.sum(objs * W, axis=-1)          # :265
    d2 = np.linalg.norm(objs - d1[..., None] * W, axis=-1)   # :268
    return d1, d2


class PBI(_Base):                           # scalarisations.py:242-273
    ID = 8

    def __init__(self, ideal_point=None, max_point=None, theta=5):
        super().__init__(ideal_point, max_point)
        self.theta = theta

    def batched(self, F, w):
        d1, d2 = _pbi_parts(self.norm(F), w)
        return d1 + self.theta * d2

    def params(self):
        return [self.theta]


class IPBI(_Base):                          # scalarisations.py:277-310
    ID = 9

    def __init__(self, ideal_point=None, max_point=None, theta=5):
        super().__init__(ideal_point, max_point)
        self.theta = theta

    def batched(self, F, w):
        d1, d2 = _pbi_parts(self.norm(F), w)
        return self.theta * d2 - d1

    def params(self):
        return [self.theta]


class QPBI(_Base):                          # scalarisations.py:314-351
    ID = 10

    def __init__(self, ideal_point=None, max_point=None, theta=5, alpha=5.0, H=5.0):
        super().__init__(ideal_point, max_point)
        self.theta, self.alpha, self.H = theta, alpha, H

    def d_star(self, k):                    # :347
        return self.alpha * (np.reciprocal(float(self.H)) * np.reciprocal(float(k)) *
                             np.sum(np.asarray(self.max_point, np.float64) - np.asarray(self.ideal_point, np.float64)))

    def batched(self, F, w):
        d1, d2 = _pbi_parts(self.norm(F), w)
        return d1 + self.theta * d2 * (d2 / self.d_star(F.shape[-1]))

    def params(self):
        return [self.theta, self.alpha, self.H]


class APD(_Base):                           # scalarisations.py:355-397
    ID = 11

    def __init__(self, ideal_point=None, max_point=None, FE=1, FE_max=10, gamma=0.010304664101210016):
        super().__init__(ideal_point, max_point)
        self.FE, self.FE_max, self.gamma = FE, FE_max, gamma

    def batched(self, F, w):
        t = self.norm(F)
        nrm = np.linalg.norm(t, axis=-1)                    # :384, before the zero fix-up
        zero = np.all(t == 0, axis=-1)
        t = np.where(zero[..., None], 1e-5, t)             # :390-391
        if np.all(w == 0):                                  # :392-393 (reference then fails for k>1)
            w = np.full_like(w, 1e-5)
        tu = t / np.linalg.norm(t, axis=-1, keepdims=True)  # :366-372
        wu = w / np.linalg.norm(w)
        theta = np.arccos(np.clip(np.sum(tu * wu, axis=-1), -1.0, 1.0))
        k = F.shape[-1]
        return (1 + k * (self.FE / self.FE_max) * (theta / self.gamma)) * nrm

    def params(self):
        return [self.FE, self.FE_max, self.gamma]


ALL = [WeightedSum, Tchebicheff, AugmentedTchebicheff, ModifiedTchebicheff, ExponentialWeightedCriterion,
       WeightedNorm, WeightedPower, WeightedProduct, PBI, IPBI, QPBI, APD]
BY_NAME = {c.__name__: c for c in ALL}
