#!/bin/bash
# Collect PMC counters for a bench workload, one counter group per rocprofv3 pass (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950; each pass stays within the per-block counter limits).
# Run from the repo root on the GPU box:  PMC_BENCH_ARGS="--config 2" bash tools/pmc_run.sh gpurun_out/pmc_c2
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="bench.py --steps 3 --warmup 1 --no-cpu-baseline ${PMC_BENCH_ARGS:-}"
i=0
# PMC_GROUPS: ';'-separated counter groups (one rocprofv3 pass each) in place of the default four;
# PMC_GROUPS=pipe: the six passes behind profiles/r05_*_pmc_pipe.json (tools/pmc_pipe.py)
PIPE_GROUPS="FETCH_SIZE;WRITE_SIZE;GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES;GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INST_CYCLES_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_ANY;GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS;TCC_HIT_sum TCC_MISS_sum"
if [ "${PMC_GROUPS:-}" = pipe ]; then PMC_GROUPS=$PIPE_GROUPS; fi
PGROUPS=${PMC_GROUPS:-"FETCH_SIZE;WRITE_SIZE;SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE;TCC_HIT_sum TCC_MISS_sum"}
IFS=';' read -r -a GROUP_LIST <<< "$PGROUPS"
for grp in "${GROUP_LIST[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$GRAFT_REPO_ROOT/$OUT" -o pass$i --output-format csv -- python3 $ARGS > "$OUT/pass$i.log" 2>&1
done
echo done
