# Round 4, call aq: the Thompson draws' split-K product with up to 32 slices of >= 96 columns (tools/ablate/varS)
# (varS kept in call ar: the zero slices skipped)
# against 16 slices of >= 256 (library): config 6 A/B twice, turbo tests on the variant, kernel stats of both.
set -e
O=gpurun_out/${1:-r04_aq}
mkdir -p $O
export TMPDIR=/tmp
cp tools/ablate/varS/liboptimobo_hip.so optimobo_amd/liboptimobo_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_turbo.py -x -q --timeout 300 --timeout-method thread > $O/turbo_tests_varS.txt 2>&1
for r in a b; do
  for v in varS prev; do
    cp tools/ablate/$v/liboptimobo_hip.so optimobo_amd/liboptimobo_hip.so
    timeout -k 10 200 python -u bench.py --config 6 --steps 100 --warmup 10 --no-cpu-baseline > $O/c6_${v}_$r.json 2>&1
  done
done
for v in varS prev; do
  cp tools/ablate/$v/liboptimobo_hip.so optimobo_amd/liboptimobo_hip.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --config 6 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_$v.log 2>&1
done
cp tools/ablate/prev/liboptimobo_hip.so optimobo_amd/liboptimobo_hip.so
echo done
