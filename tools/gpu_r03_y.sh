#!/bin/bash
# Round-3 pass Y: clock and instruction-mix counters of the GEMM shapes in tools/ablate/ablate_gemm.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_y}
mkdir -p "$O"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d "$O/pmcB" -o b --output-format csv -- ./tools/ablate/ablate_gemm > "$O/pmcB.log" 2>&1
echo pass-y-done
