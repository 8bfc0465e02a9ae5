#!/bin/bash
# Closing pass of a round on one GPU box: tools/gpu_final.sh (GPU tests, smoke, default bench, rocprofv3 stats, 2-rank
# gloo rehearsal), then configs 4 and 6 once each.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-close}
bash tools/gpu_final.sh "$(basename "$OUT")"
timeout -k 10 300 python -u bench.py --config 4 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 > "$OUT/bench_c6.json" 2> "$OUT/bench_c6.err"
echo close-done
