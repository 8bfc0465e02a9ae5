#!/bin/bash
# Steady-state runs (round 6): configs 4 and 6 with a long declared warm-up (the clocks settle over the first ~0.1-0.2 s
# of back-to-back work: profiles/r06_bb_ablate_posterior_c4_iexp.txt drifts 0.594 -> 0.555 ms over one process), each
# next to the default-warm-up run in the same call.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-steady}
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > "$OUT/bench_c4_w10.json" 2> "$OUT/bench_c4_w10.err"
timeout -k 10 300 python -u bench.py --config 4 --warmup 400 --steps 200 --no-cpu-baseline > "$OUT/bench_c4_w400.json" 2> "$OUT/bench_c4_w400.err"
timeout -k 10 300 python -u bench.py --config 4 --warmup 400 --steps 200 --no-cpu-baseline > "$OUT/bench_c4_w400b.json" 2> "$OUT/bench_c4_w400b.err"
timeout -k 10 300 python -u bench.py --config 6 --warmup 3 --steps 20 --no-cpu-baseline > "$OUT/bench_c6_w3.json" 2> "$OUT/bench_c6_w3.err"
timeout -k 10 300 python -u bench.py --config 6 --warmup 200 --steps 100 --no-cpu-baseline > "$OUT/bench_c6_w200.json" 2> "$OUT/bench_c6_w200.err"
timeout -k 10 300 python -u bench.py --warmup 30 --steps 50 --no-cpu-baseline > "$OUT/bench_c3_w30.json" 2> "$OUT/bench_c3_w30.err"
echo steady-done
