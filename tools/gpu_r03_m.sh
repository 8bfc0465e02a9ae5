#!/bin/bash
# Round-3 pass M: K block aug-r² ablation, second ordering, configs 5 and 3 shapes.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_m}
mkdir -p "$O"
timeout -k 10 150 ./tools/ablate/ablate_kblock3 1024 524288 30 > "$O/ablate_kblock3_c5.txt" 2>&1
timeout -k 10 150 ./tools/ablate/ablate_kblock3 1024 524288 30 > "$O/ablate_kblock3_c5_b.txt" 2>&1
echo pass-m-done
