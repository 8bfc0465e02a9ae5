#!/bin/bash
# Round 6: the persistent Cholesky's lookahead and far-update batching re-swept after the walker's LDS copies (§11a)
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-chol_resweep}
mkdir -p "$OUT"
timeout -k 10 400 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/chol_hybrid_sweep tools/ablate/chol_hybrid_sweep.hip
CHOL_K0S=0 CHOL_LS=2,3,1 CHOL_BW=16:4,16:3,16:5,12:4,12:3,20:4,24:4,8:3 timeout -k 10 300 ./tools/ablate/chol_hybrid_sweep 3000 > "$OUT/sweep_3000.txt" 2>&1
CHOL_K0S=0 CHOL_LS=2,3 CHOL_BW=16:4,16:3,12:4,20:4,24:4 timeout -k 10 300 ./tools/ablate/chol_hybrid_sweep 3000 2048 5000 > "$OUT/sweep_b.txt" 2>&1
echo resweep-done
