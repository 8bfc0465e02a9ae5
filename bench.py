#!/usr/bin/env python
"""Benchmark: EHVI candidate evaluations per second (BASELINE.json metric, config 3).

One step = the whole acquisition hot path over one resident batch of candidates on every
GPU, one C call (omb_eval_argmax, the fused chain): GP posterior for both objectives →
reference-mode EHVI-2D → device arg-max; then the cross-rank arg-max exchange (RCCL
all-gather of 16 B).  `--chain separate` issues the three entry points one by one
(omb_posterior, omb_ehvi2d, omb_argmax_dev); `--chain sobol` also generates the candidates
on the device inside the step (omb_eval_argmax_sobol, what the maximiser runs).  Workload per GPU: ZDT1 (n_var=6) surrogate with n_train=512 and
N = 2^20 unscrambled-Sobol candidates; rank g scores Sobol indices [g·N, (g+1)·N) (weak scaling).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N  (multi-GPU)
With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts its own N ranks (one child
process per GPU, MASTER_ADDR 127.0.0.1) before anything touches the GPU, and exits with their status.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FP64_MFMA_PEAK_TFLOPS = 78.6     # MI355X dense FP64 matrix peak (AMD spec; microbench: 70.3 measured)
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)


def zdt1(X):
    """ZDT1 (optimobo/problem.py:924-936)."""
    f1 = X[:, 0]
    g = 1 + 9.0 / (X.shape[1] - 1) * np.sum(X[:, 1:], axis=1)
    return np.column_stack([f1, g * (1 - np.sqrt(f1 / g))])


def dtlz2(X, k=3):
    """DTLZ2 with k objectives (builder-defined 3-objective workload of BASELINE config 4)."""
    g = np.sum((X[:, k - 1:] - 0.5) ** 2, axis=1)
    th = X[:, :k - 1] * np.pi / 2
    F = np.empty((len(X), k))
    for i in range(k):
        f = 1 + g
        for j in range(k - 1 - i):
            f = f * np.cos(th[:, j])
        if i > 0:
            f = f * np.sin(th[:, k - 1 - i])
        F[:, i] = f
    return F


def posterior_flops_per_candidate(n, d):
    """n(n+1) triangular L⁻¹k* + 2n ‖·‖² + 2n αᵀk* + n(2d+2) distance + ~10n Matern."""
    return n * (n + 1) + 2 * n + 2 * n + n * (2 * d + 2) + 10 * n


# BASELINE.json configs 2-5 (config 1 is the CPU-only README run).  Per-GPU candidate counts:
# configs 4 and 5 quote their totals over 8 GPUs, so one GPU scores 1/8 of them (weak scaling).
CONFIGS = {
    # BASELINE config 1: the README run end to end through the drop-in driver (host GP fit + device
    # maximiser) — reported as BO iterations/s with the time split, not a kernel benchmark
    1: dict(problem="myproblem", n=20, d=2, budget=100, acq="solve_tch"),
    # configs 2, 3 and 5 train on x_1 in [0, 1], x_2..x_d in [0, 0.3] (tail_hi): a mid-run BO state whose
    # evaluated points have drifted toward ZDT1's Pareto set (x_2..x_d = 0), so the acquisition's maximum is
    # an interior candidate; over a training set spread through [0, 1]^d the unexplored corner x = 0 (Sobol
    # index 0, ZDT1's extreme Pareto point) wins, which is also where the lowest-index tie rule lands
    2: dict(problem="zdt1", n=128, d=6, log2=16, acq="ehvi2d", tail_hi=0.3),
    3: dict(problem="zdt1", n=512, d=6, log2=20, acq="ehvi2d", tail_hi=0.3),
    # config 4's training set covers [0.5, 1]^6 (an early BO iteration: the front is still far from the
    # ideal point), so the reference's Monte-Carlo EHVI_3D is positive for ~17% of the candidates; over a
    # training set spread through [0, 1]^6 it is 0 everywhere
    4: dict(problem="dtlz2", n=256, d=6, log2=17, acq="ehvi3d", x_lo=0.5),
    5: dict(problem="zdt1", n=1024, d=30, log2=19, acq="ei_tch", tail_hi=0.3),
    # not a BASELINE config: TuRBO's Thompson-sampling step (turbo.py:75-153) — one trust region,
    # n_cand = min(100·n_var, 5000) candidates, batch_size joint posterior draws, greedy arg-mins
    6: dict(problem="zdt1", n=512, d=30, n_cand=3000, draws=64, acq="thompson"),
}
METRIC = "EHVI candidate evals/sec at n_train=512, 2-obj; 1/2/4/8-GPU scaling"


def setup_problem(n, d, seed=0, problem="zdt1", x_lo=0.0, tail_hi=1.0):
    """Training set of a BASELINE config: n points uniform in [x_lo, 1]^d (numpy default_rng(seed)), the
    coordinates x_2..x_d then scaled by tail_hi, the problem's objectives, ARD length scales ℓ_j ~ U[0.2, 2]
    (default_rng(seed + 1)), σ_f² = Var(Y_k)."""
    rng = np.random.default_rng(seed)
    X = rng.uniform(x_lo, 1.0, (n, d))
    X[:, 1:] *= tail_hi
    Y = zdt1(X) if problem == "zdt1" else dtlz2(X)
    ls = np.random.default_rng(seed + 1).uniform(0.2, 2.0, d)
    variances = [float(np.var(Y[:, o])) for o in range(Y.shape[1])]
    return X, Y, ls, variances


def candidates(d, start, count):
    from scipy.stats import qmc
    s = qmc.Sobol(d=d, scramble=False)
    if start:
        s.fast_forward(start)
    return s.random(count)


def blas_threads():
    """Threads the numpy BLAS actually runs with (threadpoolctl), and the host's logical CPU count."""
    try:
        from threadpoolctl import threadpool_info
        threads = max([p.get("num_threads", 1) for p in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        threads = 1
    return int(threads), int(os.cpu_count() or 1)


def cpu_baseline(X, targets, ls, variances, Xc, acq_fn, label, seconds):
    """The oracle (numpy fp64, batched, BLAS-threaded) on a bounded sample of the same workload:
    oracle posterior (GPy restatement, dtrtrs) for every surrogate → ``acq_fn(mu, var)`` → arg-max,
    in chunks of 4096 candidates for about ``seconds`` seconds."""
    from oracle import acquisition as oacq
    from oracle import gp as ogp
    threads, ncpu = blas_threads()
    gps = [ogp.ExactGP(X, targets[:, o], ls, variances[o]) for o in range(targets.shape[1])]
    chunk = 4096
    done = 0
    t0 = time.perf_counter()
    while done < len(Xc):                 # a prefix of the batch: never past its end
        xc = Xc[done: done + chunk]
        mus, vs = [], []
        for g in gps:
            m, v = g.predict(xc)
            mus.append(m[:, 0])
            vs.append(v[:, 0])
        oacq.argmax(acq_fn(np.array(mus), np.array(vs)))
        done += len(xc)
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    # the box gives one GPU's job a share of the host's CPUs (OMP_NUM_THREADS; 16 on this pool), and numpy's
    # BLAS runs with that many threads: `cores`.  per_core and the host-wide figure (the rate scaled linearly to
    # all of os.cpu_count(), an upper bound: BLAS-2 dtrtrs does not scale linearly) are reported beside it.
    rate = done / dt
    return {"value": rate, "unit": "candidates/s", "cores": threads, "host_cpu_count": ncpu, "kind": "port",
            "per_core": rate / max(threads, 1), "host_linear_upper_bound": rate / max(threads, 1) * ncpu,
            "sample": f"the first {done} of the {len(Xc)} candidates of this GPU's batch in chunks of {chunk}; "
                      f"oracle posterior (dtrtrs) + {label} + arg-max, {dt:.1f} s; cores = numpy BLAS threads "
                      f"used (threadpoolctl; the job's CPU share)"}


def run_solve(args, cfg, world_size, rank):
    """README MyProblem (README.md:28-45): MultiSurrogateOptimiser + Tchebicheff, budget 100,
    n_init 20, sample_exponent 3, timed end to end with the fit / maximiser split."""
    import torch
    import optimobo_amd.algorithms.optimisers as opti
    import optimobo_amd.scalarisations as sc
    from optimobo_amd.problem import ElementwiseProblem

    class MyProblem(ElementwiseProblem):
        def __init__(self):
            super().__init__(n_var=2, n_obj=2, xl=np.array([-2, -2]), xu=np.array([2, 2]))

        def _evaluate(self, x, out, *a, **k):
            out["F"] = [100 * (x[0] ** 2 + x[1] ** 2), (x[0] - 1) ** 2 + x[1] ** 2]

    budget = args.steps if args.steps != 50 else cfg["budget"]
    np.random.seed(0)
    opt = opti.MultiSurrogateOptimiser(MyProblem(), [0, 0], [700, 12], seed=1)
    split = {"fit": 0.0, "maximise": 0.0}

    def timed(name, fn):
        def w(*a, **k):
            t = time.perf_counter()
            r = fn(*a, **k)
            torch.cuda.synchronize()
            split[name] += time.perf_counter() - t
            return r
        return w
    opt._fit_many = timed("fit", opt._fit_many)          # the per-objective fits (concurrent on the GPU)
    opt._maximise = timed("maximise", opt._maximise)
    t0 = time.perf_counter()
    res = opt.solve(budget=budget, n_init_samples=20, sample_exponent=3,
                    acquisition_func=sc.Tchebicheff([0, 0], [700, 12]))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if rank == 0:
        print(json.dumps({
            "metric": "README MyProblem MultiSurrogateOptimiser.solve() BO iterations/sec (BASELINE config 1)",
            "value": budget / el, "unit": "iterations/s", "n_gpus": 1, "steps": budget, "warmup": 0,
            "ms_per_step": el / budget * 1e3, "higher_is_better": True, "scaling": "none", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic",
            "config": {"workload": "README MyProblem (2-var, 2-obj), Tchebicheff expected decomposition, budget "
                                   f"{budget}, n_init 20, sample_exponent 3, {opt.n_candidates} device candidates "
                                   f"x {opt.refine_rounds + 1} rounds per iteration", "parallelism": "dp1"},
            "split_s": {"gp_fit": split["fit"], "device_maximiser": split["maximise"],
                        "other": el - split["fit"] - split["maximise"]},
            "final_hv": float(res.hypervolume_convergence[-1]), "n_evaluations": int(len(res.ysample)),
            "roofline": None, "cpu_baseline": reference_solve_c1(),
        }))


def thompson_flops(n, N, B):
    """Algorithmic flops of one Thompson step: V = L⁻¹K* (triangular, n²N), Σ = K** − VᵀV (lower
    triangle, nN(N+1)), Cholesky N³/3, draws L·z (triangular, B·N²); kernel evaluations not counted."""
    return n * n * N + n * N * (N + 1) + N ** 3 / 3.0 + B * N * N


def cpu_thompson(X, yagg, ls, var, Xc, B, seconds):
    """The reference's own recipe on the host: GPy full-covariance predict (oracle restatement) +
    numpy.random.multivariate_normal (SVD, as GPy's posterior_samples_f) + greedy arg-mins."""
    from oracle import gp as ogp
    from oracle import turbo as oturbo
    cores, ncpu = blas_threads()
    g = ogp.ExactGP(X, yagg, ls, var)
    steps = 0
    t0 = time.perf_counter()
    while True:
        mu, cov = g.predict_full_cov(Xc)
        y = np.random.default_rng(steps).multivariate_normal(mu, cov, B, method="svd")
        oturbo.select(y.T[:, None, :])
        steps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": steps * len(Xc) / dt, "unit": "candidates/s", "cores": int(cores), "host_cpu_count": ncpu,
            "kind": "port",
            "sample": f"{steps} Thompson step(s) of {len(Xc)} candidates x {B} draws (oracle full-cov posterior "
                      f"+ numpy multivariate_normal (SVD) + greedy arg-min), {dt:.1f} s"}


def run_thompson(args, cfg, world_size, rank, device, backend):
    """TuRBO Thompson step per GPU: omb_posterior_samples + omb_thompson_select (synchronous)."""
    import torch
    import torch.distributed as dist
    from optimobo_amd import scalarisations as sc
    from optimobo_amd.device import AcqContext
    from optimobo_amd.gp import GPState

    n, d, N, B = cfg["n"], cfg["d"], cfg["n_cand"], cfg["draws"]
    X, Y, ls, _ = setup_problem(n, d, problem=cfg["problem"])
    tch = sc.Tchebicheff(Y.min(axis=0), Y.max(axis=0))
    yagg = tch(Y, np.array([0.5, 0.5]))
    var = float(np.var(yagg))
    ctx = AcqContext(device.index)
    if args.chol_mode is not None:
        ctx.debug_set("chol_mode", args.chol_mode)
    if args.cov_fused is not None:
        ctx.debug_set("cov_fused", args.cov_fused)
    if args.syrk_glds is not None:
        ctx.debug_set("syrk_glds", args.syrk_glds)
    ctx.set_gp_state(0, GPState(X, yagg, ls, var))
    rng = np.random.default_rng(100 + rank)
    # a trust region of side 0.2 around a training point (turbo.py:82-111), one per rank
    centre = X[rank % n]
    Xc_host = np.clip(centre + 0.2 * (rng.uniform(0, 1, (N, d)) - 0.5), 0, 1)
    Xc = torch.as_tensor(Xc_host, device=device)
    Z = torch.as_tensor(rng.standard_normal((B, N)), device=device)
    Yd = torch.empty((B, N), dtype=torch.float64, device=device)
    idx = torch.empty(B, dtype=torch.int64, device=device)
    jit = [0.0]

    def step():
        _, jit[0] = ctx.posterior_samples(0, Xc, Z, out=Yd)
        ctx.thompson_select(Yd, out=idx)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world_size > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world_size > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world_size > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    step_ms = elapsed / args.steps * 1e3
    fl = thompson_flops(n, N, B)
    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline:
        cpu = cpu_thompson(X, yagg, ls, var, Xc_host, B, args.cpu_seconds)
    if rank == 0:
        out = {
            "metric": "TuRBO Thompson-sampling candidate evals/sec (joint posterior draws + greedy arg-min)",
            "value": N * world_size * args.steps / elapsed,
            "unit": "candidates/s", "n_gpus": world_size, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": step_ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"TuRBO Thompson step, ZDT1 Tchebicheff surrogate, n_train={n}, n_var={d}, "
                                   f"n_cand={N} (min(100*n_var, 5000)), {B} joint draws, one trust region per GPU",
                       "n_train": n, "n_var": d, "n_cand": N, "draws": B, "global_batch": N * world_size,
                       "parallelism": f"dp{world_size}"},
            "roofline": {"bound": "mfma", "achieved": fl / (step_ms * 1e-3) / 1e12, "peak": FP64_MFMA_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": fl / (step_ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS,
                         "traffic": None,
                         "kernel": "whole step (covariance GEMMs + blocked Cholesky + draws + select); "
                                   "algorithmic flops per step = n^2 N + n N (N+1) + N^3/3 + B N^2",
                         "ms_per_launch": step_ms},
            "cpu_baseline": cpu, "jitter": jit[0],
        }
        print(json.dumps(out))
    if world_size > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


def reference_cpu(config):
    """The reference's own per-candidate path timed in the build container (tools/ref_cpu_baseline.py,
    committed as profiles/r02_ref_cpu_baseline.jsonl): 1 thread, as differential_evolution calls it."""
    path = os.path.join(REPO, "profiles", "r02_ref_cpu_baseline.jsonl")
    try:
        with open(path) as f:
            recs = [json.loads(line) for line in f if line.strip()]
    except (OSError, ValueError):
        return None
    for r in recs:
        if r.get("config") == config:
            return {"value": r["value"], "unit": r["unit"], "cores": r["cores"], "kind": "reference",
                    "what": r["what"], "measured_in": "build container (8 vCPU Xeon), tools/ref_cpu_baseline.py",
                    "source": "profiles/r02_ref_cpu_baseline.jsonl"}
    return None


def reference_solve_c1():
    """The reference's own MultiSurrogateOptimiser.solve on the README run, timed in the build container
    (tools/ref_solve_baseline.py → profiles/r03_ref_solve_c1.json; GPy / pymoo replaced by doubles)."""
    for name in ("r04_ref_solve_c1.json", "r03_ref_solve_c1.json"):
        path = os.path.join(REPO, "profiles", name)
        try:
            with open(path) as f:
                r = json.loads(f.read().strip().splitlines()[-1])
            break
        except (OSError, ValueError, IndexError):
            r = None
    if r is None:
        return None
    return {"value": r["value"], "unit": r["unit"], "cores": r["cores"], "kind": "reference",
            "sample": f"the whole run (budget 100, {r['seconds']:.0f} s, final HV {r['final_hv']:.2f}); "
                      + r["doubles"],
            "measured_in": r.get("measured_in", "build container (8 vCPU Xeon)") + ", tools/ref_solve_baseline.py; "
                           "GPy and pymoo are absent there and replaced by the doubles named in `sample`",
            "source": f"profiles/{name}"}


def load_traffic(n, N, kernel="posterior"):
    """HBM bytes per launch of the posterior ("posterior") or K-block ("kblock") kernel from the
    committed rocprofv3 PMC summary (profiles/traffic.json, tools/pmc_summary.py), if present."""
    path = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
        key = f"{kernel}_n{n}_N{N}"
        return t.get(key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def load_pipe(config, kernel):
    """FP64-pipe occupancy of a kernel from the committed PMC summaries (tools/pmc_pipe.py): round 6's
    (profiles/r06_v_pmc_pipe.json: configs 3 and 4 after their occupancy changes) first, then round 5's
    (profiles/r05_zm_pmc_pipe.json): MFMA-busy and VALU-issue fractions per SIMD (they never co-execute on gfx950),
    or None."""
    for name in ("r06_v_pmc_pipe.json", "r05_zm_pmc_pipe.json"):
        path = os.path.join(REPO, "profiles", name)
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        for k, v in t.items():
            if f"pmc_c{config}:" in k and kernel in k:
                return {x: v[x] for x in ("mfma_busy_frac", "valu_issue_frac", "fp64_pipe_busy_frac") if x in v} | \
                    {"source": f"profiles/{name} (rocprofv3 --pmc, separate passes)"}
    return None


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n):
    """`python bench.py --gpus N` without a launcher: start N ranks of this script as child processes with
    torch.distributed.run's environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT) and wait for them.
    Runs before torch is imported, so this process never touches the GPU.  If one rank fails, the others
    (which would wait in a collective) are terminated; the exit status is the first failure's, else 0."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                for q in live:
                    q.terminate()
        time.sleep(0.1)
    return status


def launch_check(world_size, rank, backend):
    """--launch-check: the rank set-up alone (process group, one all-gather of the ranks), no GPU work with
    gloo.  Rank 0 prints what torch.distributed saw."""
    import torch
    import torch.distributed as dist
    dist.init_process_group(backend=backend, init_method="env://")
    dev = "cpu" if backend == "gloo" else torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    mine = torch.tensor([rank], dtype=torch.int64, device=dev)
    got = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(got, mine)
    if rank == 0:
        print(json.dumps({"launch_check": True, "world_size": dist.get_world_size(), "backend": dist.get_backend(),
                          "ranks": [int(t.item()) for t in got], "master_addr": os.environ.get("MASTER_ADDR")}))
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS), help="BASELINE.json config")
    ap.add_argument("--log2-cand", type=int, default=None, help="candidates per GPU = 2^this (default: config)")
    ap.add_argument("--mode", default="reference", choices=["reference", "textbook"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kblock", action="store_true")
    ap.add_argument("--chain", default="fused", choices=["fused", "separate", "sobol"])
    ap.add_argument("--stage-timing", action="store_true", help="events around every stage (adds ~5 us/stage)")
    ap.add_argument("--timing-stride", type=int, default=None,
                    help="record the timing events on every s-th step of the timed loop only (each record adds "
                         "~2.5 us of GPU time to its step: config 2 82.8 us per step with events on every step, "
                         "77.3-77.8 on every 8th, gpurun_out/r04_ae).  Default: from the warm-up's step length, "
                         "1 for steps >= 1 ms (configs 3-5: 2.5 us is < 0.05%%), else 8")
    ap.add_argument("--one-launch", type=int, default=None, choices=[0, 1, 2],
                    help="omb_debug_set(FUSED_CHAIN): 0 EHVI-2D and the arg-max as separate launches, 1 as one "
                         "ticketed launch, 2 EHVI-2D reducing to per-workgroup pairs + the arg-max's second pass "
                         "(default: the library's)")
    ap.add_argument("--argmax-passes", type=int, default=None, choices=[1, 2],
                    help="omb_debug_set(ARGMAX_PASSES): the arg-max as one launch or two (default: the library's, 2)")
    ap.add_argument("--chol-mode", type=int, default=None, choices=[0, 1, 2, 4, 5, 6, 8, 10, 12, 14],
                    help="omb_debug_set(CHOL_MODE): Cholesky auto / per-step launches / one persistent launch; + 4: "
                         "with release-acquire hand-offs")
    ap.add_argument("--syrk-glds", type=int, default=None, choices=[0, 1],
                    help="omb_debug_set(SYRK_GLDS): the covariance SYRK's three-stage direct-to-LDS operand pipeline "
                         "(config 6; default: the library's, 1)")
    ap.add_argument("--cov-fused", type=int, default=None, choices=[0, 1],
                    help="omb_debug_set(COV_FUSED): K(X*, X*) in the covariance SYRK's epilogue (config 6; default: "
                         "the library's, 1)")
    ap.add_argument("--uniform-train", action="store_true",
                    help="train on X uniform in [0, 1]^d (SURVEY 8d) instead of the config's mid-run BO box "
                         "(configs 2-5); the step's work is the same, the arg-max lands on the unexplored corner")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks and the process group only, print what torch.distributed saw")
    ap.add_argument("--cache-seed", type=int, default=1,
                    help="Sobol seed of the MC sample cache (optimisers.py:121-141, unseeded in the reference). "
                         "1: s01 = +0.070, reference-mode EHVI positive where it improves (default); "
                         "0: s01 = -0.028, reference-mode EHVI <= 0 everywhere (degenerate arg-max)")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))          # no launcher: this process starts the ranks

    import torch
    import torch.distributed as dist

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world_size != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world_size}")
    # OMB_DIST_BACKEND=gloo rehearses the multi-rank path on a box with fewer GPUs than ranks
    # (ranks then share GPUs round-robin); the driver's multi-GPU runs use nccl (= RCCL).
    backend = os.environ.get("OMB_DIST_BACKEND", "nccl")
    if args.launch_check:
        return launch_check(world_size, rank, backend)
    gpu = local_rank % max(1, torch.cuda.device_count()) if backend == "gloo" else local_rank
    dist_info = {"backend": None, "world_size": 1}
    if world_size > 1:
        torch.cuda.set_device(gpu)
        dist.init_process_group(backend=backend, init_method="env://")
        dist_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                     "rccl_version": ".".join(map(str, torch.cuda.nccl.version())) if dist.get_backend() == "nccl"
                     else None}
        if "OMB_DIST_BACKEND" not in os.environ:
            assert dist_info["backend"] == "nccl", f"multi-GPU bench must run over RCCL, got {dist_info['backend']}"
        assert dist_info["world_size"] == world_size
    device = torch.device("cuda", gpu)
    local_rank = gpu

    if cfg["acq"] == "thompson":
        return run_thompson(args, cfg, world_size, rank, device, backend)
    if cfg["acq"] == "solve_tch":
        return run_solve(args, cfg, world_size, rank)

    from optimobo_amd import pareto
    from optimobo_amd import scalarisations as sc
    from optimobo_amd.device import AcqContext
    from optimobo_amd.gp import GPState
    from optimobo_amd.parallel import global_argmax

    n, d, acq_kind = cfg["n"], cfg["d"], cfg["acq"]
    N = 1 << (args.log2_cand if args.log2_cand is not None else cfg["log2"])
    if args.uniform_train:                           # SURVEY §8(d)'s training set: X uniform in [0, 1]^d
        cfg = {k: v for k, v in cfg.items() if k not in ("x_lo", "tail_hi")}
    X, Y, ls, variances = setup_problem(n, d, problem=cfg["problem"], x_lo=cfg.get("x_lo", 0.0),
                                        tail_hi=cfg.get("tail_hi", 1.0))
    k_obj = Y.shape[1]
    pf = pareto.calc_pf(Y)
    r = Y.max(axis=0) + 0.1 * (Y.max(axis=0) - Y.min(axis=0))
    cache = pareto.cached_samples(k_obj, 5, seed=args.cache_seed)

    ctx = AcqContext(local_rank)
    if args.one_launch is not None:
        ctx.debug_set("fused_chain", args.one_launch)
    if args.argmax_passes is not None:
        ctx.debug_set("argmax_passes", args.argmax_passes)
    if args.chol_mode is not None:
        ctx.debug_set("chol_mode", args.chol_mode)
    if acq_kind == "ei_tch":
        # ParEGO-style mono surrogate: Tchebicheff-aggregate the objectives (parego.py:212-219)
        tch = sc.Tchebicheff(Y.min(axis=0), Y.max(axis=0))
        yagg = tch(Y, np.array([0.5, 0.5]))
        states = [GPState(X, yagg, ls, float(np.var(yagg)))]
        best_y = float(yagg.min())
    else:
        states = [GPState(X, Y[:, o], ls, variances[o]) for o in range(k_obj)]
    n_obj = len(states)
    for o, st in enumerate(states):
        ctx.set_gp_state(o, st)

    start = rank * N
    Xc_host = candidates(d, start, N)
    Xc = torch.as_tensor(Xc_host, device=device)
    mu = torch.empty((n_obj, N), dtype=torch.float64, device=device)
    var = torch.empty_like(mu)
    acq = torch.empty(N, dtype=torch.float64, device=device)
    raised = torch.empty(N, dtype=torch.int32, device=device)
    pair = torch.empty(2, dtype=torch.float64, device=device)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if acq_kind == "ehvi2d":
        s00, s01 = pareto.cache_stats(cache)
        pf_dev = torch.as_tensor(pareto.stripes_2d(pf), device=device)
    elif acq_kind == "ehvi3d":
        hv_pf = pareto.hypervolume(pf, r)
        coords, _, boxes = pareto.box_decomposition(pf, r)
        cache_dev = torch.as_tensor(cache, device=device)

    # the plan of the fused chain: the same acquisition as acquisition() below
    if acq_kind == "ehvi2d":
        ctx.plan_ehvi2d(pareto.stripes_2d(pf), r, s00, s01, mode=args.mode)
    elif acq_kind == "ehvi3d" and args.mode == "textbook":
        ctx.plan_ehvi_boxes(coords, boxes)       # exact EHVI, box decomposition staged in LDS
    elif acq_kind == "ehvi3d":
        ctx.plan_ehvi3d_mc(cache, r, hv_pf)
    else:
        ctx.plan_ei(best_y, 1e-6)
    if args.chain == "sobol":
        # unscrambled Sobol over [0, 1]^d: the same points as `candidates` above
        ctx.set_sobol(d, np.zeros(d), np.ones(d), scramble=False)

    def acquisition():
        if acq_kind == "ehvi2d":
            ctx.ehvi2d(mu, var, pf_dev, r, s00, s01, mode=args.mode, out=acq)
        elif acq_kind == "ehvi3d" and args.mode == "textbook":
            ctx.ehvi_boxes(mu, var, coords, boxes, out=acq)
        elif acq_kind == "ehvi3d":
            ctx.ehvi3d_mc(mu, var, cache_dev, r, hv_pf, out=acq, raised=raised)
        else:
            ctx.ei(mu[0], var[0], best_y, 1e-6, out=acq)

    def step(i=None):
        if args.chain == "fused":
            ctx.eval_argmax(Xc, offset=start, out=pair)
        elif args.chain == "sobol":
            ctx.eval_argmax_sobol(start, N, out=pair)
        else:
            if i is not None:
                ev[i][0].record()
            ctx.posterior(Xc, n_obj, out=(mu, var))
            if i is not None:
                ev[i][1].record()
            acquisition()
            ctx.argmax_dev(acq, offset=start, out=pair)
        return global_argmax(pair)

    torch.cuda.synchronize()
    t_w = time.perf_counter()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    warm_ms = (time.perf_counter() - t_w) / args.warmup * 1e3 if args.warmup else None
    stride = args.timing_stride
    if stride is None:            # every launch when an event pair is noise against the step
        stride = 1 if warm_ms is None or warm_ms >= 1.0 else 8

    if world_size > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == 1 and args.chain != "separate":
            # HIP events on the chain's stream: around the posterior (level 1) or every stage (2).  Switched on
            # after step 0 is queued: step 0 follows the synchronize on an idle GPU and is not a steady-state
            # launch, so the average covers steps 1, 1 + stride, ...
            ctx.debug_set("timing_stride", stride)
            ctx.timing(2 if args.stage_timing else 1)
        best = step(i if i >= 1 else None)
    torch.cuda.synchronize()
    if world_size > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stage_ms = None
    chains = args.steps
    if args.chain != "separate" and args.steps > 1:
        stage_sum, chains = ctx.timing_read()
        ctx.timing(0)
        stage_ms = {k: v / chains for k, v in stage_sum.items() if args.stage_timing or k == "posterior"}
    elif args.chain != "separate":
        stage_ms, chains = {"posterior": float("nan")}, 0
    if world_size > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if stage_ms is not None:
        post_ms = stage_ms["posterior"] if chains else float("nan")
    else:
        post_ms = float(np.mean([a.elapsed_time(b) for a, b in ev[1:]])) if args.steps > 1 else float("nan")
        chains = max(args.steps - 1, 0)
    best = best.cpu().numpy()

    # standalone K(X, X*) block: the HBM-bound kernel of the north star
    kblock = None
    if not args.no_kblock:
        K = torch.empty((n, N), dtype=torch.float64, device=device)
        ctx.kernel_block(0, Xc, out=K)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            ctx.kernel_block(0, Xc, out=K)
        e1.record()
        torch.cuda.synchronize()
        kb_ms = e0.elapsed_time(e1) / reps
        kb_bytes = 8.0 * (n + d) * N + 8.0 * n * (d + 1)      # 8(n+d) per candidate + model state
        # the same launch against the FP64 pipe: distance n(2d+2) + ~10n Matern flop per candidate (SURVEY §8d's
        # posterior count without the triangular product); at n_var > 8 the cross-term MFMAs + transform, not the
        # stores, bound it
        kb_flops = float(n) * (2 * d + 2 + 10) * N
        kb_fp64 = kb_flops / (kb_ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS
        kblock = {"bound": "hbm" if d <= 8 else "mfma",   # n_var > 8: the FP64 pipe (cross-term MFMAs + Matern VALU)
                  "achieved": kb_bytes / (kb_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": kb_bytes / (kb_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": load_traffic(n, N, "kblock"),
                  "fp64_frac": kb_fp64, "fp64_tflops": kb_flops / (kb_ms * 1e-3) / 1e12,
                  "ms": kb_ms,
                  "pipe": load_pipe(args.config, "kernel_block"),
                  "note": f"omb_kernel_block writes K ({n}, {N}) fp64 to HBM; frac = HBM fraction, fp64_frac = "
                          f"{n * (2 * d + 12)} flop per candidate / time / {FP64_MFMA_PEAK_TFLOPS} TFLOP/s; pipe = the "
                          f"FP64 pipe's MFMA + VALU occupancy from PMC (the Matern transform's VALU work and the "
                          f"cross-term MFMAs share it)"}
        del K

    # per-iteration model-state install, outside `value`: what a BO iteration does before its
    # batch — factorise Ky on the device and install (α, L⁻¹) for every objective (omb_gp_fit_state)
    from optimobo_amd.gp import DeviceGPState
    dev_states = [DeviceGPState(st.X, st.y, st.lengthscale, st.variance) for st in states]
    for o, st in enumerate(dev_states):
        ctx.set_gp_state(o, st)
    torch.cuda.synchronize()
    t_up = time.perf_counter()
    reps_up = 5
    for _ in range(reps_up):
        for o, st in enumerate(dev_states):
            ctx.set_gp_state(o, st)
    torch.cuda.synchronize()
    state_ms = (time.perf_counter() - t_up) / reps_up * 1e3

    flops = n_obj * posterior_flops_per_candidate(n, d) * N
    achieved = flops / (post_ms * 1e-3) / 1e12
    step_ms = elapsed / args.steps * 1e3
    # the posterior is one launch inside every step, so its event-timed average cannot exceed the step
    check = bool(post_ms <= step_ms)
    roofline = {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / FP64_MFMA_PEAK_TFLOPS, "traffic": load_traffic(n, N),
                "kernel": f"posterior_kernel (omb_posterior, {n_obj} objective(s), n_train={n}, n_var={d})",
                "ms_per_launch": post_ms,
                "launches_timed": int(chains),
                "pipe": load_pipe(args.config, "posterior_kernel"),
                "timing_stride": stride,
                "check": check,
                "timing": "HIP events on the chain's stream around the posterior launch"
                          + (f" of every {stride}th timed step from step 1" if args.chain != "separate"
                             and stride > 1 else " of every timed step but the first")}

    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline:
        from oracle import acquisition as oacq
        if acq_kind == "ehvi2d":
            cpu = cpu_baseline(X, Y, ls, variances, Xc_host,
                               lambda m, v: oacq.ehvi2d(m, v, pf, r, cache, mode=args.mode),
                               f"{args.mode}-mode EHVI-2D", args.cpu_seconds)
        elif acq_kind == "ehvi3d" and args.mode == "reference":
            def mc3(m, v):
                val, raised = oacq.ehvi3d_reference(m, v, hv_pf, r, cache)
                return np.where(raised, np.nan, val)
            cpu = cpu_baseline(X, Y, ls, variances, Xc_host, mc3, "reference Monte-Carlo EHVI-3D", args.cpu_seconds)
        elif acq_kind == "ehvi3d":
            from oracle import pareto as opar
            lo_b, hi_b = opar.nondominated_boxes(pf, r)
            cpu = cpu_baseline(X, Y, ls, variances, Xc_host, lambda m, v: oacq.ehvi_exact_boxes(m, v, lo_b, hi_b),
                               "exact EHVI-3D over the box decomposition", args.cpu_seconds)
        else:
            cpu = cpu_baseline(X, yagg[:, None], ls, [states[0].variance], Xc_host,
                               lambda m, v: oacq.ei(m[0], v[0], best_y, 1e-6), "ParEGO EI (var + 1e-6)",
                               args.cpu_seconds)

    if rank == 0:
        total = N * world_size * args.steps
        ehvi3d_label = ("3-obj EHVI (reference Monte-Carlo form)" if args.mode == "reference"
                        else "3-obj exact EHVI (box decomposition in LDS)")
        label = {"ehvi2d": f"2-obj EHVI ({args.mode} mode)", "ehvi3d": ehvi3d_label,
                 "ei_tch": "ParEGO Tchebicheff EI (mono surrogate)"}[acq_kind]
        out = {
            "metric": METRIC if args.config == 3 else f"{label} candidate evals/sec (BASELINE config {args.config})",
            "value": total / elapsed,
            "unit": "candidates/s",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{label}, {cfg['problem'].upper()} surrogate, n_train={n}, n_var={d}, "
                                   f"2^{int(np.log2(N))} Sobol candidates per GPU (BASELINE config {args.config})",
                       "n_train": n, "n_var": d, "n_obj": k_obj, "candidates_per_gpu": N,
                       "global_batch": N * world_size, "parallelism": f"dp{world_size}"},
            "roofline": roofline,
            "roofline_kblock": kblock,
            "cpu_baseline": cpu,
            "reference_cpu_per_candidate": reference_cpu(args.config),
            "chain": args.chain,
            "stage_ms": stage_ms,
            "state_install_ms": state_ms,
            "best": {"value": float(best[0]), "index": int(best[1]),
                     "x": candidates(d, int(best[1]), 1)[0].tolist() if best[1] >= 0 else None},
            "distributed": dict(dist_info, candidates_per_rank=N, rank_shard=f"Sobol indices [r*{N}, (r+1)*{N})",
                                collective="all_gather of one 16-B {value, index} pair per step"),
            "cache": {"seed": args.cache_seed, "samples": int(cache.shape[0])},
        }
        if acq_kind == "ehvi2d":
            out["cache"].update(s00=s00, s01=s01)
        if acq_kind == "ehvi2d" and args.mode == "reference" and s01 < 0:
            out["best"]["note"] = ("reference-mode EHVI passes sigma_B = var_0*s01 (util_functions.py:163-167); this "
                                   f"cache has s01 = {s01:.4g} < 0, so the acquisition is <= 0 everywhere and the "
                                   "arg-max is the lowest index among its maxima (DESIGN.md section 2, quirk 2)")
        out["config"]["train_box"] = f"[0, 1]^{d} (uniform, SURVEY 8d)"
        if "x_lo" in cfg:
            out["config"]["train_box"] = f"[{cfg['x_lo']}, 1]^{d}"
        if "tail_hi" in cfg:
            out["config"]["train_box"] = f"x_1 in [0, 1], x_2..x_{d} in [0, {cfg['tail_hi']}]"
        print(json.dumps(out), flush=True)
    if world_size > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()
    if not check:
        raise SystemExit(f"bench.py: roofline check failed: posterior {post_ms:.4f} ms per launch > "
                         f"{step_ms:.4f} ms per step (the event timing is not measuring the launch)")


if __name__ == "__main__":
    main()
