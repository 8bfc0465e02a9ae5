#!/bin/bash
# Round-end style pass on one GPU box: GPU tests, smoke, default bench, rocprofv3 kernel stats of the
# default bench, and a 2-rank gloo rehearsal of the multi-rank bench path (ranks share the one GPU).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final}
mkdir -p "$OUT"
bash tools/gpu_verify.sh "$(basename "$OUT")"
OMB_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-kblock \
  > "$OUT/bench_gloo2.json" 2> "$OUT/bench_gloo2.err"
echo final-done
