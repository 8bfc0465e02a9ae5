# Round 4, call x: the default Cholesky (per-step launches, then the persistent launch for the last 32 steps):
# sweep with the library rule (k0 = -1) and neighbours, check tool, full Cholesky / TuRBO / GP-fit tests, config 6.
set -e
O=gpurun_out/${1:-r04_x}
mkdir -p $O
export TMPDIR=/tmp
CHOL_K0S=-1,0,8,16,40,56 timeout -k 10 200 ./tools/ablate/chol_hybrid_sweep 512 1000 2100 3000 4097 5000 > $O/sweep.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_turbo.py tests/test_gpu_gpfit.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
for m in 1 0; do
  timeout -k 10 200 python -u bench.py --config 6 --steps 20 --warmup 5 --no-cpu-baseline --chol-mode $m > $O/bench_c6_m$m.json 2>&1
done
echo done
