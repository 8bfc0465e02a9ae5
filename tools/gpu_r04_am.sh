# Round 4, call am: EHVI-2D with one lane per candidate for batches >= 2^19 (two for >= 2^18, four below):
# parity / fused / workload / edge tests, then configs 3 and 2 A/B against the previous commit's library
# (tools/ablate/prev, swapped on the box's copy only), rocprofv3 stats of config 3.
set -e
O=gpurun_out/${1:-r04_am}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_properties.py tests/test_gpu_fused.py tests/test_gpu_bench_workloads.py tests/test_gpu_edges.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
cp optimobo_amd/liboptimobo_hip.so $O/../new_lib.so.tmp
for r in a b; do
  cp $O/../new_lib.so.tmp optimobo_amd/liboptimobo_hip.so
  timeout -k 10 200 python -u bench.py --config 3 --steps 30 --warmup 5 --no-cpu-baseline --no-kblock > $O/c3_new_$r.json 2>&1
  timeout -k 10 200 python -u bench.py --config 2 --steps 400 --warmup 40 --no-cpu-baseline --no-kblock > $O/c2_new_$r.json 2>&1
  cp tools/ablate/prev/liboptimobo_hip.so optimobo_amd/liboptimobo_hip.so
  timeout -k 10 200 python -u bench.py --config 3 --steps 30 --warmup 5 --no-cpu-baseline --no-kblock > $O/c3_prev_$r.json 2>&1
  timeout -k 10 200 python -u bench.py --config 2 --steps 400 --warmup 40 --no-cpu-baseline --no-kblock > $O/c2_prev_$r.json 2>&1
done
cp $O/../new_lib.so.tmp optimobo_amd/liboptimobo_hip.so
rm -f $O/../new_lib.so.tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kblock > $O/prof.log 2>&1
echo done
