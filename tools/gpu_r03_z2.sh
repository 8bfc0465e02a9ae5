#!/bin/bash
# Round-3 pass Z2: blocked Cholesky built with and without VGPR-form MFMA, interleaved on one box.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03_z2}
mkdir -p "$O"
for i in 1 2; do
  timeout -k 10 180 ./tools/ablate/ablate_chol 512 3000 5000 > "$O/chol_vgpr_$i.txt" 2>&1
  timeout -k 10 180 ./tools/ablate/ablate_chol_agpr 512 3000 5000 > "$O/chol_agpr_$i.txt" 2>&1
done
echo pass-z2-done
