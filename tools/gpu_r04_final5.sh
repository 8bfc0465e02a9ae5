# Round 4 closing pass on the final tree (after the draws' split-K change): GPU suite, smoke, default bench,
# rocprofv3 stats (tools/gpu_verify.sh), then configs 6 and 2 (400 steps).  The first failing step ends it.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_final5}
mkdir -p "$OUT"
bash tools/gpu_verify.sh "$(basename "$OUT")"
timeout -k 10 300 python -u bench.py --config 6 > "$OUT/bench_c6.json" 2> "$OUT/bench_c6.err"
timeout -k 10 300 python -u bench.py --config 2 --steps 400 --warmup 40 > "$OUT/bench_c2_400.json" 2> "$OUT/bench_c2.err"
echo final-done
