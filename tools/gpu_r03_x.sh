#!/bin/bash
# Round-3 pass X: PMC counters of the SYRK/NN GEMM shapes (library kernel vs rocBLAS) in tools/ablate/ablate_gemm.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_x}
mkdir -p "$O"
timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d "$O/pmcA" -o a --output-format csv -- ./tools/ablate/ablate_gemm > "$O/pmcA.log" 2>&1
echo pass-x-done
