# Round 4, call aj: persistent Cholesky workers draw their next ticket when a task starts and poll a task's flags
# (Measured slower and reverted; see DESIGN §9a "Worker latency".)
# together: check tool (bitwise vs per-step, watchdog), phases at N = 3000, hybrid k0 sweep, turbo tests, config 6
# A/B against the previous commit's library (tools/ablate/prev, swapped on the box's copy only).
set -e
O=gpurun_out/${1:-r04_aj}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ablate/chol_persist_check 65536 130 200 1000 2000 3000 3500 5000 > $O/check.txt 2>&1
timeout -k 10 60 ./tools/ablate/chol_persist_check_nodbg 65536 3000 > $O/check_timed.txt 2>&1
CHOL_K0S=0,4,8,11,15,20 timeout -k 10 200 ./tools/ablate/chol_hybrid_sweep 1000 3000 5000 > $O/sweep.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_turbo.py -x -q --timeout 300 --timeout-method thread > $O/turbo_tests.txt 2>&1
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
