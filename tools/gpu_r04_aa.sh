# Round 4, call aa: EHVI-2D with φ from exp_nonpos and 1/σ multiplies: parity / properties / fused / workload tests,
# configs 2 and 3.
set -e
O=gpurun_out/${1:-r04_aa}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_properties.py tests/test_gpu_fused.py tests/test_gpu_bench_workloads.py tests/test_gpu_edges.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
timeout -k 10 200 python -u bench.py --config 2 --steps 200 --warmup 20 --no-cpu-baseline --stage-timing > $O/bench_c2_stages.json 2>&1
timeout -k 10 200 python -u bench.py --config 2 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_c2.json 2>&1
timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3.json 2>&1
echo done
