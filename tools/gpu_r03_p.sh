#!/bin/bash
# Round-3 pass P: diagonal block factored by one wave (OMB_CHOL_1W) vs four, traced, N = 512 / 3000 / 5000.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_p}
mkdir -p "$O"
timeout -k 10 120 ./tools/ablate/ablate_chol 512 3000 5000 > "$O/ablate_chol_4w.txt" 2>&1
timeout -k 10 120 ./tools/ablate/ablate_chol_1w 512 3000 5000 > "$O/ablate_chol_1w.txt" 2>&1
echo pass-p-done
