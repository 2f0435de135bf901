#!/usr/bin/env bash
# One parameterised GPU job for gpurun (replaces the per-call scripts): every argument is one recipe,
# run in order under its own time limit; the job stops at the first failure (abort, fault, timeout).
#
#   tools/gpu.sh <out-subdir> "<recipe> [args...]" ["<recipe> [args...]" ...]
#
# recipes (logs / results land in gpurun_out/<out-subdir>/):
#   tests <name> <pytest args...>   python -m pytest -m gpu <args> (per-test timeout 120 s, step limit 600 s)
#   testsl <name> <pytest args...>  the same with an 1100 s step limit (the whole suite)
#   bench <name> <bench.py args...> bench.py ... --json-out <name>.json
#   prof  <name> <bench.py args...> rocprofv3 --kernel-trace --stats around bench.py, reduced to <name>_kernels.csv
#   proftrace <name> <bench.py args...> the same, plus the raw kernel trace as <name>_trace.csv.gz
#   py    <name> <script args...>   python <script> <args>
#   pylong <name> <script args...>  the same with an 1100 s step limit
#   pyprof <name> <script args...>  rocprofv3 --kernel-trace --stats around python3 <script> <args>
#   smoke                           __graft_entry__.smoke()
# Leading KEY=VALUE tokens after <name> are exported for that step only, e.g. "bench b2 GAI_X=1 --steps 2".
# e.g. /usr/local/graft/bin/gpurun --timeout 900 -- tools/gpu.sh r3a "tests kern tests/test_kernels_gpu.py" \
#        "bench b1 --steps 3 --warmup 1"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH=$PWD
export TMPDIR=/tmp
O=$PWD/gpurun_out/$1; shift; mkdir -p "$O"

step() {  # step SECONDS LOG cmd...
  local secs=$1 log=$2; shift 2
  # heartbeat into the log: a long quiet step (multi-rank tests, pytest -q) is not mistaken for a hang;
  # the step's own timeout still bounds it
  : > "$log"
  ( while sleep 50; do echo "[gpu.sh] heartbeat $(date +%T)" >> "$log"; done ) &
  local hb=$!
  env "${envs[@]}" timeout -k 10 "$secs" "$@" >> "$log" 2>&1
  local rc=$?
  kill $hb 2>/dev/null; wait $hb 2>/dev/null
  echo "[gpu.sh] rc=$rc cmd=$*" >> "$log"
  tail -4 "$log"
  return $rc
}

for spec in "$@"; do
  read -r -a a <<< "$spec"
  r=${a[0]}; n=${a[1]:-x}; rest=("${a[@]:2}")
  envs=()
  while [ ${#rest[@]} -gt 0 ] && [[ ${rest[0]} == *=* ]] && [[ ${rest[0]} != -* ]]; do envs+=("${rest[0]}"); rest=("${rest[@]:1}"); done
  echo "[gpu.sh] $(date +%T) $spec"
  case $r in
    tests) step 600 "$O/$n.log" python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread \
             -p no:cacheprovider "${rest[@]}"
           rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;  # test failures (1) do not stop the job
    testsl) step 1100 "$O/$n.log" python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread \
             -p no:cacheprovider "${rest[@]}"
           rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;  # the whole suite, as the driver runs it
    bench) step 600 "$O/$n.log" python bench.py "${rest[@]}" --json-out "$O/$n.json" || exit $? ;;
    prof)  rm -rf "/tmp/prof_$n"
           step 600 "$O/$n.log" rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/prof_$n" -o run -- \
             python3 "$PWD/bench.py" "${rest[@]}" --json-out "$O/$n.json" || exit $?
           python tools/rocprof_summary.py "/tmp/prof_$n/**/*kernel_stats.csv" -o "$O/${n}_kernels.csv" --top 60 \
             > /dev/null || exit $?
           python tools/trace_gaps.py "/tmp/prof_$n/**/*kernel_trace.csv" --from-frac 0.6 --top 40 \
             -o "$O/${n}_gaps.json" > /dev/null || exit $? ;;
    proftrace) rm -rf "/tmp/prof_$n"  # prof + the raw kernel trace (gzipped) for gap analysis
           step 600 "$O/$n.log" rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/prof_$n" -o run -- \
             python3 "$PWD/bench.py" "${rest[@]}" --json-out "$O/$n.json" || exit $?
           python tools/rocprof_summary.py "/tmp/prof_$n/**/*kernel_stats.csv" -o "$O/${n}_kernels.csv" --top 60 \
             > /dev/null || exit $?
           f=$(find "/tmp/prof_$n" -name "*kernel_trace.csv" | head -1); gzip -c "$f" > "$O/${n}_trace.csv.gz" || exit $? ;;
    py)    step 600 "$O/$n.log" python "${rest[@]}" || exit $? ;;
    pylong) step 1100 "$O/$n.log" python "${rest[@]}" || exit $? ;;  # long runs (1M-chunk ingest)
    pyprof) rm -rf "/tmp/prof_$n"
           step 600 "$O/$n.log" rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/prof_$n" -o run -- \
             python3 "${rest[@]}" || exit $?
           python tools/rocprof_summary.py "/tmp/prof_$n/**/*kernel_stats.csv" -o "$O/${n}_kernels.csv" --top 60 \
             > /dev/null || exit $?
           python tools/rocprof_summary.py "/tmp/prof_$n/**/*kernel_trace.csv" --by-grid -o "$O/${n}_grid.csv" \
             --top 80 > /dev/null || exit $? ;;
    smoke) step 300 "$O/smoke.log" python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $? ;;
    *) echo "unknown recipe $r"; exit 2 ;;
  esac
done
echo "[gpu.sh] done"
