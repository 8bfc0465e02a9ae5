"""Das-Dennis reference directions (pymoo ``get_reference_directions("das-dennis", k, n_partitions)``),
used by the optimisers to draw a random weight vector each iteration (optimisers.py:182,234)."""
from itertools import combinations

import numpy as np


def das_dennis(n_dim, n_partitions):
    """All points of the simplex lattice {w ≥ 0, Σw = 1, w·n_partitions ∈ ℕ}: C(p+k-1, k-1) rows."""
    if n_partitions == 0:
        return np.full((1, n_dim), 1.0 / n_dim)
    rows = []
    # stars and bars: choose k-1 bar positions among p+k-1 slots
    for bars in combinations(range(n_partitions + n_dim - 1), n_dim - 1):
        prev, parts = -1, []
        for b in bars:
            parts.append(b - prev - 1)
            prev = b
        parts.append(n_partitions + n_dim - 1 - prev - 1)
        rows.append(parts)
    return np.asarray(rows, dtype=np.float64) / n_partitions


def get_reference_directions(name, n_dim, n_partitions=None, **kwargs):
    if name not in ("das-dennis", "uniform"):
        raise ValueError(f"unsupported reference-direction scheme {name!r}")
    return das_dennis(n_dim, n_partitions)
