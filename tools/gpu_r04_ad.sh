# Round 4, call ad: EHVI-2D reducing to per-workgroup pairs + the arg-max's second pass (fused_chain 2) against the
# separate launches (0) and the ticketed one launch (1, now with a grid of at most 1024 workgroups): tests, A/B/C
# twice at config 2, config 3 once each, kernel durations of mode 2.
set -e
O=gpurun_out/${1:-r04_ad}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_bench_workloads.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
for r in a b; do
  for m in 0 2 1; do
    timeout -k 10 200 python -u bench.py --config 2 --steps 400 --warmup 40 --no-cpu-baseline --no-kblock --one-launch $m > $O/c2_m${m}_$r.json 2>&1
  done
done
for m in 0 2 1; do
  timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline --no-kblock --one-launch $m > $O/c3_m$m.json 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_m2 -o run -- python3 bench.py --config 2 --steps 200 --warmup 20 --no-cpu-baseline --no-kblock --one-launch 2 > $O/prof_m2.log 2>&1
echo done
