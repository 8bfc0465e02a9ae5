#!/bin/bash
# Every bench configuration once (GPU box): BASELINE configs 1-5 and the TuRBO config 6.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-benchall}
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --config 3 > "$OUT/c3.json" 2> "$OUT/c3.err"
timeout -k 10 300 python -u bench.py --config 2 > "$OUT/c2.json" 2> "$OUT/c2.err"
timeout -k 10 300 python -u bench.py --config 4 > "$OUT/c4_mc.json" 2> "$OUT/c4_mc.err"
timeout -k 10 300 python -u bench.py --config 4 --mode textbook > "$OUT/c4_exact.json" 2> "$OUT/c4_exact.err"
timeout -k 10 300 python -u bench.py --config 5 > "$OUT/c5.json" 2> "$OUT/c5.err"
timeout -k 10 300 python -u bench.py --config 6 --steps 10 --warmup 2 > "$OUT/c6.json" 2> "$OUT/c6.err"
timeout -k 10 600 python -u bench.py --config 1 > "$OUT/c1.json" 2> "$OUT/c1.err"
echo bench-all-done
