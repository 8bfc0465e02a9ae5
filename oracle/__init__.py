"""CPU oracle for the OptiMOBO acquisition hot path — TEST INFRASTRUCTURE ONLY.

This package is the parity checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may import it.
The shipped path (``optimobo_amd``) never imports anything from here and fails loudly
when its HIP library is missing.

Every function is a numpy fp64 restatement of the reference algorithm and cites the
reference ``file:line`` it follows (paths relative to aje220/OptiMOBO v0.2.1).

Pinning:
  * acquisition arithmetic (EHVI-2D, EHVI-3D MC, HV-PoI, expected decomposition, the
    twelve scalarisations, EI, 2-D cell decomposition) is pinned against golden vectors
    produced by the reference's own functions (``tests/golden/make_golden.py``);
  * GP posterior arithmetic lives in GPy (absent here, ``gpy>=1.10``); it is restated
    from GPy's published formulas and pinned against an independent implementation,
    scikit-learn 1.7.2 ``GaussianProcessRegressor`` (golden vectors in the same fixtures).
"""
