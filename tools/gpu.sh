#!/bin/bash
# One parameterised GPU-box step runner (replaces the per-call one-off scripts of rounds 1-4).
# Every GPU step runs under its own time limit; the first failing step ends the call (set -e).
#
#   bash tools/gpu.sh OUT STEP [STEP ...]
#
# OUT is a directory under gpurun_out/.  Each STEP is one quoted word list:
#   "bench NAME ARGS..."   python bench.py ARGS > OUT/NAME.json (stderr OUT/NAME.err)
#   "prof NAME ARGS..."    rocprofv3 --kernel-trace --stats of bench.py ARGS (OUT/NAME/…, line in OUT/NAME.json)
#   "pmc NAME ARGS..."     PMC passes (tools/pmc_run.sh) of bench.py ARGS into OUT/NAME
#   "test NAME PYTEST..."  python -m pytest -m gpu PYTEST > OUT/NAME.txt
#   "testk NAME K1,K2 FILES..."  the same with -k "K1 or K2" (commas: a step is split on whitespace)
#   "smoke"                __graft_entry__.smoke() > OUT/smoke.txt
#   "py NAME SCRIPT ARGS..." python -u SCRIPT ARGS > OUT/NAME.txt
#   "bin NAME SECS EXE ARGS..." a built tool binary under timeout SECS > OUT/NAME.txt
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
for step in "$@"; do
  set -- $step
  kind=$1
  shift
  echo "[$(date +%T)] $kind $*"
  case $kind in
    bench)
      name=$1; shift
      timeout -k 10 400 python -u bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
      tail -c 600 "$OUT/$name.json" ;;
    prof)
      name=$1; shift
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/$name" -o run \
        --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" ;;
    pmc)
      name=$1; shift
      PMC_BENCH_ARGS="$*" bash tools/pmc_run.sh "$OUT/$name" ;;
    test)
      name=$1; shift
      timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
        > "$OUT/$name.txt" 2>&1
      tail -3 "$OUT/$name.txt" ;;
    testk)
      name=$1; kexpr=${2//,/ or }; shift 2
      timeout -k 10 1000 python -u -m pytest -m gpu --maxfail 20 -v --timeout 300 --timeout-method thread -k "$kexpr" "$@" \
        > "$OUT/$name.txt" 2>&1
      tail -3 "$OUT/$name.txt" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1
      cat "$OUT/smoke.txt" ;;
    py)
      name=$1; shift
      timeout -k 10 600 python -u "$@" > "$OUT/$name.txt" 2>&1 ;;
    bin)
      name=$1; secs=$2; shift 2
      timeout -k 10 "$secs" "$@" > "$OUT/$name.txt" 2>&1 ;;
    *)
      echo "unknown step $kind"; exit 2 ;;
  esac
done
echo "gpu.sh done"
