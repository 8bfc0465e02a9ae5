"""Problem definition surface (optimobo/problem.py:14-656), without pymoo.

Users subclass ``Problem`` (vectorised ``_evaluate(X, out)`` on (N, n_var)) or
``ElementwiseProblem`` (``_evaluate(x, out)`` per row) and optionally
``_evaluate_constraints``.  ``evaluate(x)`` on a 1-D x returns the (n_obj,) objective vector
the optimisers consume (optimisers.py:59, 176, 256); on (N, n_var) it returns (N, n_obj).
Runners (looped, starmap, dask, joblib, ray) evaluate elementwise problems as in the
reference (problem.py:42-130).
"""
from abc import abstractmethod
from functools import wraps

import numpy as np


# ----------------------------------------------------------------------------- element runners
class ElementwiseEvaluationFunction:
    def __init__(self, problem, args, kwargs):
        self.problem, self.args, self.kwargs = problem, args, kwargs

    def __call__(self, x):
        out = {}
        self.problem._evaluate(x, out, *self.args, **self.kwargs)
        return out


class ElementwiseEvaluationFunctionConstraint(ElementwiseEvaluationFunction):
    def __call__(self, x):
        out = {}
        self.problem._evaluate_constraints(x, out, *self.args, **self.kwargs)
        return out


class LoopedElementwiseEvaluation:
    def __call__(self, f, X):
        return [f(x) for x in X]


class StarmapParallelization:
    def __init__(self, starmap):
        self.starmap = starmap

    def __call__(self, f, X):
        return list(self.starmap(f, [[x] for x in X]))

    def __getstate__(self):
        return {k: v for k, v in self.__dict__.items() if k != "starmap"}


class DaskParallelization:
    def __init__(self, client):
        self.client = client

    def __call__(self, f, X):
        return [job.result() for job in [self.client.submit(f, x) for x in X]]

    def __getstate__(self):
        return {k: v for k, v in self.__dict__.items() if k != "client"}


class JoblibParallelization:
    def __init__(self, aJoblibParallel, aJoblibDelayed, *args, **kwargs):
        self.parallel, self.delayed = aJoblibParallel, aJoblibDelayed

    def __call__(self, f, X):
        return self.parallel(self.delayed(f)(x) for x in X)

    def __getstate__(self):
        return {k: v for k, v in self.__dict__.items() if k not in ("parallel", "delayed")}


class RayParallelization:
    def __init__(self, job_resources=None):
        try:
            import ray  # noqa: F401
        except ImportError as e:  # pragma: no cover - ray is optional
            raise AssertionError('Ray must be installed! `pip install -U "ray[default]"`') from e
        self.job_resources = job_resources or {"num_cpus": 1}

    def __call__(self, f, X):  # pragma: no cover - ray is optional
        import ray
        runnable = ray.remote(f.__call__.__func__).options(**self.job_resources)
        return ray.get([runnable.remote(f, x) for x in X])


# ----------------------------------------------------------------------------- helpers
def default_shape(problem, n):
    v = problem.n_var
    return dict(F=(n, problem.n_obj), G=(n, problem.n_ieq_constr), H=(n, problem.n_eq_constr),
                dF=(n, problem.n_obj, v), dG=(n, problem.n_ieq_constr, v), dH=(n, problem.n_eq_constr, v))


def _cached(fn):
    """pymoo's @Cache: memoise a no-argument-dependent problem property."""
    attr = "__cache_" + fn.__name__

    @wraps(fn)
    def wrapper(self, *args, **kwargs):
        if attr not in self.__dict__:
            self.__dict__[attr] = fn(self, *args, **kwargs)
        return self.__dict__[attr]
    return wrapper


def _as_rows(X):
    """pymoo at_least_2d_array(X, extend_as='row', return_if_reshaped=True)."""
    X = np.asarray(X)
    if X.ndim == 1:
        return X[None, :], True
    return X, False


# ----------------------------------------------------------------------------- Problem
class Problem:
    def __init__(self, n_var=-1, n_obj=1, n_ieq_constr=0, n_eq_constr=0, xl=None, xu=None, vtype=None, vars=None,
                 elementwise=False, elementwise_func=ElementwiseEvaluationFunction,
                 elementwise_func_constr=ElementwiseEvaluationFunctionConstraint,
                 elementwise_runner=None, requires_kwargs=False, replace_nan_values_by=None,
                 exclude_from_serialization=None, callback=None, strict=True, **kwargs):
        self.n_var = n_var
        self.n_obj = n_obj
        self.n_ieq_constr = max(n_ieq_constr, kwargs["n_constr"]) if "n_constr" in kwargs else n_ieq_constr
        self.n_eq_constr = n_eq_constr
        self.data = dict(**kwargs)
        self.xl, self.xu = xl, xu
        self.callback = callback
        if vars is not None:
            self.vars = vars
            self.n_var = len(vars)
            if self.xl is None:
                self.xl = {k: getattr(v, "lb", None) for k, v in vars.items()}
            if self.xu is None:
                self.xu = {k: getattr(v, "ub", None) for k, v in vars.items()}
        self.vtype = vtype
        self.elementwise = elementwise
        self.elementwise_func = elementwise_func
        self.elementwise_func_constr = elementwise_func_constr
        self.elementwise_runner = elementwise_runner if elementwise_runner is not None else LoopedElementwiseEvaluation()
        self.requires_kwargs = requires_kwargs
        self.strict = strict
        if n_var > 0:
            if self.xl is not None:
                self.xl = (self.xl if isinstance(self.xl, np.ndarray) else np.ones(n_var) * self.xl).astype(float)
            if self.xu is not None:
                self.xu = (self.xu if isinstance(self.xu, np.ndarray) else np.ones(n_var) * self.xu).astype(float)
        self.replace_nan_values_by = replace_nan_values_by
        self.exclude_from_serialization = exclude_from_serialization

    # -- shared evaluation machinery (objectives and constraints)
    def _run(self, X, return_values_of, return_as_dictionary, args, kwargs, constraints):
        if not self.requires_kwargs:
            kwargs = {}
        if isinstance(X, np.ndarray) and X.dtype != object:
            X, single = _as_rows(X)
            assert X.shape[1] == self.n_var, f"Input dimension {X.shape[1]} are not equal to n_var {self.n_var}!"
        else:
            single = not isinstance(X, (list, np.ndarray))
        raw = (self.do_constraints if constraints else self.do)(X, return_values_of, *args, **kwargs)
        out = {}
        for key, val in raw.items():
            val = np.array(val)
            if single:
                val = val[0]
            if self.replace_nan_values_by is not None:
                val[np.isnan(val)] = self.replace_nan_values_by
            try:
                out[key] = val.astype(np.float64)
            except (TypeError, ValueError):
                out[key] = val
        if self.callback is not None:
            self.callback(X, out)
        if return_as_dictionary:
            return out
        if len(return_values_of) == 1:
            return out[return_values_of[0]]
        return tuple(out[k] for k in return_values_of)

    def evaluate(self, X, *args, return_values_of=None, return_as_dictionary=False, **kwargs):
        return self._run(X, return_values_of or ["F"], return_as_dictionary, args, kwargs, constraints=False)

    def evaluate_constraints(self, X, *args, return_values_of=None, return_as_dictionary=False, **kwargs):
        if return_values_of is None:
            return_values_of = (["G"] if self.n_ieq_constr > 0 else []) + (["H"] if self.n_eq_constr > 0 else [])
        return self._run(X, return_values_of, return_as_dictionary, args, kwargs, constraints=True)

    def _dispatch(self, X, out, args, kwargs, constraints):
        if self.elementwise:
            maker = self.elementwise_func_constr if constraints else self.elementwise_func
            for elem in self.elementwise_runner(maker(self, args, kwargs), X):
                for k, v in elem.items():
                    if out.get(k) is None:
                        out[k] = []
                    out[k].append(v)
            for k in out:
                if out[k] is not None:
                    out[k] = np.array(out[k])
        elif constraints:
            self._evaluate_constraints(X, out, *args, **kwargs)
        else:
            self._evaluate(X, out, *args, **kwargs)

    def do(self, X, return_values_of, *args, **kwargs):
        out = {name: None for name in return_values_of}
        self._dispatch(X, out, args, kwargs, constraints=False)
        return self._format_dict(out, len(X), return_values_of)

    def do_constraints(self, X, return_values_of, *args, **kwargs):
        out = {name: None for name in return_values_of}
        self._dispatch(X, out, args, kwargs, constraints=True)
        return self._format_dict(out, len(X), return_values_of)

    def _format_dict(self, out, N, return_values_of):
        shape = default_shape(self, N)
        ret = {}
        for name, v in out.items():
            if v is None:
                continue
            if name in shape:
                if isinstance(v, list):
                    v = np.column_stack(v)
                try:
                    v = v.reshape(shape[name])
                except Exception as e:
                    raise Exception(f"Problem Error: {name} can not be set, expected shape {shape[name]} "
                                    f"but provided {v.shape}", e)
            ret[name] = v
        for name in return_values_of:
            if name not in ret:
                ret[name] = np.full(shape.get(name, N), np.inf)
        return ret

    # -- pymoo-style known-front helpers
    @_cached
    def nadir_point(self, *args, **kwargs):
        pf = self.pareto_front(*args, **kwargs)
        return None if pf is None else np.max(pf, axis=0)

    @_cached
    def ideal_point(self, *args, **kwargs):
        pf = self.pareto_front(*args, **kwargs)
        return None if pf is None else np.min(pf, axis=0)

    @_cached
    def pareto_front(self, *args, **kwargs):
        pf = self._calc_pareto_front(*args, **kwargs)
        if pf is None:
            return None
        pf = np.atleast_2d(pf)
        if pf.shape[1] == 2:
            pf = pf[np.argsort(pf[:, 0])]
        return pf

    @_cached
    def pareto_set(self, *args, **kwargs):
        ps = self._calc_pareto_set(*args, **kwargs)
        return None if ps is None else np.atleast_2d(ps)

    @property
    def n_constr(self):
        return self.n_ieq_constr + self.n_eq_constr

    @abstractmethod
    def _evaluate(self, x, out, *args, **kwargs):
        pass

    @abstractmethod
    def _evaluate_constraints(self, x, out, *args, **kwargs):
        pass

    def has_bounds(self):
        return self.xl is not None and self.xu is not None

    def has_constraints(self):
        return self.n_constr > 0

    def bounds(self):
        return self.xl, self.xu

    def name(self):
        return self.__class__.__name__

    def _calc_pareto_front(self, *args, **kwargs):
        return None

    def _calc_pareto_set(self, *args, **kwargs):
        return None

    def __str__(self):
        return (f"# name: {self.name()}\n# n_var: {self.n_var}\n# n_obj: {self.n_obj}\n"
                f"# n_ieq_constr: {self.n_ieq_constr}\n# n_eq_constr: {self.n_eq_constr}\n")

    def __getstate__(self):
        if self.exclude_from_serialization is None:
            return self.__dict__
        state = self.__dict__.copy()
        for key in self.exclude_from_serialization:
            state[key] = None
        return state


class ElementwiseProblem(Problem):
    def __init__(self, elementwise=True, **kwargs):
        super().__init__(elementwise=elementwise, **kwargs)
