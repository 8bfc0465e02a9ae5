# Round 4, call j: r² upper clamp (degenerate lengthscale) pinned; table README run; fused/one-launch tests;
# Cholesky stress; EHVI+argmax one launch (cheap ticket) vs separate on configs 2/3; config 4 after the clamp.
set -e
O=gpurun_out/${1:-r04_j}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_cov_table.py -x -v -s -k "sweep or degenerate or readme_run" --timeout 300 --timeout-method thread > $O/cov_table.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 240 --timeout-method thread > $O/fused_tests.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_turbo.py -x -q -k stress --timeout 240 --timeout-method thread > $O/chol_stress.txt 2>&1
for v in 0 1; do
  timeout -k 10 200 python -u bench.py --config 2 --steps 200 --warmup 20 --no-cpu-baseline --one-launch $v > $O/bench_c2_ol$v.json 2>&1
  timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline --one-launch $v > $O/bench_c3_ol$v.json 2>&1
done
timeout -k 10 200 python -u bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c4.json 2>&1
echo done
