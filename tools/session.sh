#!/bin/bash
# One GPU-box session as a list of steps; every GPU step runs under its own time limit
# and the session stops at the first failure (no retries).
#   usage: bash tools/session.sh <tag> <step>...
# steps (outputs under gpurun_out/<tag>/):
#   tests[=<pytest -k expr>]      the -m gpu tests (commas for spaces)   pytest.log
#   bench=<workload>[,<args>]     one bench line (args: comma-separated)  bench_<workload>[args].json
#   smoke                         __graft_entry__.smoke()                  smoke.log
#   stats=<workload>[,<args>]     rocprofv3 kernel trace + stats          <workload>[args]_kernel_stats.csv
#   pmc=<workload>                FETCH / WRITE / TCC hit-miss passes     pmc<k>_<workload>/
#   deep=<workload>[,<packets>[,<v>]]  SQ / TA / TCP counter passes (v: an _ab/ library)  deep_<workload>[_<v>]/
#   cal                           the random-line FETCH_SIZE calibration  pmc_cal/
#   ab=<workload>,<v>[,<v>...]    timing-only A/B of library variants (v = main or a
#                                 directory under _ab/ holding libcilium_hip.so)  ab_<workload>_<v>/
#   env=<workload>,<ENV=V ...>    kernel trace of a short bench run under the settings
#   abx=<v>,<workload>[,<args>]   kernel trace of a short bench run (args) with library variant v
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # run <seconds> <log> <cmd>...: one limited step, the session ends on failure
  local lim=$1 log=$2; shift 2
  echo "[$(date +%T)] $*" >&2
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[session] rc=$rc: $*" >&2; tail -20 "$log" >&2; exit $rc; fi
}
kstats() {
  python3 - "$1" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith(("void cv::", "cv::")):
        print(f"  {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4}  {r['Name'][:70]}")
PY
}
for st in "$@"; do
  name=${st%%=*}; arg=""; [ "$name" != "$st" ] && arg=${st#*=}
  IFS=, read -r -a A <<< "$arg"
  case $name in
  tests)
    K=(); [ -n "$arg" ] && K=(-k "${arg//,/ }")   # (commas stand for spaces)
    run 900 "$OUT/pytest.log" python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "${K[@]}"
    grep -cE "PASSED" "$OUT/pytest.log" >&2 ;;
  bench)
    W=${A[0]}; T=$W; [ ${#A[@]} -gt 1 ] && T=${W}$(printf '%s' "${A[@]:1}" | tr -c 'a-zA-Z0-9.' '_')
    echo "[$(date +%T)] bench $W ${A[*]:1}" >&2
    timeout -k 10 600 python3 -u bench.py --workload "$W" "${A[@]:1}" > "$OUT/bench_$T.json" 2> "$OUT/bench_$T.err" \
      || { rc=$?; echo "[session] bench rc=$rc" >&2; tail -20 "$OUT/bench_$T.err" >&2; exit $rc; }
    cat "$OUT/bench_$T.json" ;;
  smoke)
    run 300 "$OUT/smoke.log" python3 -c "import __graft_entry__ as g; g.smoke()"
    tail -1 "$OUT/smoke.log" >&2 ;;
  stats)
    W=${A[0]}; T=$W; [ ${#A[@]} -gt 1 ] && T=${W}$(printf '%s' "${A[@]:1}" | tr -c 'a-zA-Z0-9.' '_')
    run 600 "$OUT/stats_$T.log" rocprofv3 --kernel-trace --stats -d "$OUT/stats_$T" -o run --output-format csv \
      -- python3 bench.py --workload "$W" --steps 10 --warmup 2 --no-cpu "${A[@]:1}"
    cp "$OUT/stats_$T/run_kernel_stats.csv" "$OUT/${T}_kernel_stats.csv"
    echo "== $T" >&2; kstats "$OUT/${T}_kernel_stats.csv" >&2 ;;
  pmc)
    W=${A[0]}; i=0
    for CTRS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      run 240 "$OUT/pmc${i}_$W.log" rocprofv3 --pmc $CTRS -d "$OUT/pmc${i}_$W" -o run --output-format csv \
        -- python3 bench.py --workload "$W" --steps 3 --warmup 1 --no-cpu
    done ;;
  deep)
    W=${A[0]}; P=${A[1]:-4194304}; V=${A[2]:-}; i=0
    if [ -n "$V" ]; then export CV_LIB=$PWD/_ab/$V/libcilium_hip.so; D=deep_${W}_$V; else unset CV_LIB; D=deep_$W; fi
    for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
                "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_WAIT_ANY" \
                "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"; do
      i=$((i+1))
      mkdir -p "$OUT/$D"
      run 150 "$OUT/$D/p$i.log" rocprofv3 --pmc $CTRS -d "$OUT/$D/p$i" -o run --output-format csv \
        -- python3 bench.py --workload "$W" --packets "$P" --steps 1 --warmup 1 --no-cpu
    done
    unset CV_LIB
    python3 tools/pmc_table.py "$OUT/$D" > "$OUT/$D.txt" 2>&1 ;;
  cal)
    run 120 "$OUT/pmc_cal.log" rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_cal" -o run --output-format csv \
      -- python3 tools/pmc_calibrate.py ;;
  ab)
    W=${A[0]}
    for v in "${A[@]:1}"; do
      if [ "$v" = main ]; then L=$PWD/cilium_amd/_lib/libcilium_hip.so; else L=$PWD/_ab/$v/libcilium_hip.so; fi
      k=$(ls -d "$OUT/ab_${W}_$v"* 2>/dev/null | wc -l); D=$OUT/ab_${W}_$v$([ "$k" -gt 0 ] && echo ".$k")
      CV_LIB=$L run 300 "$D.log" rocprofv3 --kernel-trace --stats -d "$D" -o run --output-format csv \
        -- python3 bench.py --workload "$W" --steps 5 --warmup 1 --no-cpu
      echo "== $v" >&2; kstats "$D/run_kernel_stats.csv" >&2
    done ;;
  abx)                                  # abx=<v>,<workload>[,<args>]: kernel trace of a bench run with a library variant
    v=${A[0]}; W=${A[1]}
    if [ "$v" = main ]; then L=$PWD/cilium_amd/_lib/libcilium_hip.so; else L=$PWD/_ab/$v/libcilium_hip.so; fi
    T=${W}$(printf '%s' "${A[@]:2}" | tr -c 'a-zA-Z0-9.' '_')
    k=$(ls -d "$OUT/abx_${v}_$T"* 2>/dev/null | wc -l); D=$OUT/abx_${v}_$T$([ "$k" -gt 0 ] && echo ".$k")
    CV_LIB=$L run 400 "$D.log" rocprofv3 --kernel-trace --stats -d "$D" -o run --output-format csv \
      -- python3 bench.py --workload "$W" --steps 5 --warmup 1 --no-cpu "${A[@]:2}"
    echo "== $v $T: $(grep -o '"value": [0-9.]*' "$D.log" | head -1)" >&2; kstats "$D/run_kernel_stats.csv" >&2 ;;
  env)
    W=${A[0]}
    k=$(ls -d "$OUT"/env* 2>/dev/null | wc -l)
    env ${A[@]:1} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/env$k" -o run --output-format csv \
      -- python3 bench.py --workload "$W" --steps 5 --warmup 1 --no-cpu > "$OUT/env$k.log" 2>&1 \
      || { rc=$?; echo "[session] env rc=$rc" >&2; tail -20 "$OUT/env$k.log" >&2; exit $rc; }
    echo "== env$k: ${A[*]:1}" >&2; kstats "$OUT/env$k/run_kernel_stats.csv" >&2 ;;
  *) echo "unknown step $st" >&2; exit 2 ;;
  esac
done
exit 0
