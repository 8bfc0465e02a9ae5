#!/bin/bash
# Round-3 pass G: config-2 posterior ablation (prefetch), PMC passes for configs 4 and 5.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_g}
mkdir -p "$O"
timeout -k 10 150 ./tools/ablate/ablate_posterior 128 65536 6 2 > "$O/ablate_c2.txt" 2>&1
PMC_BENCH_ARGS="--config 4" bash tools/pmc_run.sh "$O/pmc_c4"
PMC_BENCH_ARGS="--config 5" bash tools/pmc_run.sh "$O/pmc_c5"
echo pass-g-done
