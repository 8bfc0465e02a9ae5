# Round 4 final pass: GPU tests, smoke, default bench (config 3 with the CPU baseline) + kernel stats, configs 1,
# 2, 4, 5, 6 lines, PMC passes for configs 3 and 5 (posterior and K block traffic).  The first failing step ends it.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_final}
mkdir -p "$OUT"
bash tools/gpu_verify.sh "$(basename "$OUT")"
for c in 2 4 5 6; do
  timeout -k 10 300 python -u bench.py --config $c > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"
done
timeout -k 10 400 python -u bench.py --config 1 > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err"
PMC_BENCH_ARGS="--config 3" bash tools/pmc_run.sh "$OUT/pmc_c3" > "$OUT/pmc_c3.log" 2>&1
PMC_BENCH_ARGS="--config 5" bash tools/pmc_run.sh "$OUT/pmc_c5" > "$OUT/pmc_c5.log" 2>&1
echo final-done
