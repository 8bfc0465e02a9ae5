#!/bin/bash
# n ≤ 128 register-resident posterior: where the time goes (staging, generation, transform) at 2^16 and 2^18
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r02_v46}
mkdir -p "$O"
timeout -k 10 120 ./tools/ablate/ablate_posterior 128 65536 6 2 > "$O/ablate_c2.txt" 2>&1
timeout -k 10 120 ./tools/ablate/ablate_posterior 128 262144 6 2 > "$O/ablate_c2_N18.txt" 2>&1
echo v46-done
