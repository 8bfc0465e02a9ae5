# Round 4, call af: Thompson step with the draws queued before the Cholesky status is read (status copied into
# pinned memory) against the previous commit's library (tools/ablate/prev, swapped in on the box's copy only):
# turbo tests, config 6 A/B/A/B.
set -e
O=gpurun_out/${1:-r04_af}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_turbo.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
cp optimobo_amd/liboptimobo_hip.so $O/../new_lib.so.tmp
for r in a b; do
  cp $O/../new_lib.so.tmp optimobo_amd/liboptimobo_hip.so
  timeout -k 10 200 python -u bench.py --config 6 --steps 100 --warmup 10 --no-cpu-baseline > $O/c6_new_$r.json 2>&1
  cp tools/ablate/prev/liboptimobo_hip.so optimobo_amd/liboptimobo_hip.so
  timeout -k 10 200 python -u bench.py --config 6 --steps 100 --warmup 10 --no-cpu-baseline > $O/c6_prev_$r.json 2>&1
done
cp $O/../new_lib.so.tmp optimobo_amd/liboptimobo_hip.so
rm -f $O/../new_lib.so.tmp
echo done
