#!/bin/bash
# timing-only A/B of library variants on config 3 (variants may give wrong answers)
#   usage: bash tools/ab_run.sh <tag> <variant>...   (variant "main" = cilium_amd/_lib)
T=$1; shift
OUT=gpurun_out/$T; mkdir -p $OUT; export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = main ]; then L=/root/repo/cilium_amd/_lib/libcilium_hip.so; else L=/root/repo/_ab/$v/libcilium_hip.so; fi
  echo "== $v $(date +%T)"
  CV_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run --output-format csv \
     -- python3 bench.py --workload ${W:-config3} --steps 5 --warmup 1 --no-cpu > $OUT/$v.log 2>&1 || { echo "fail $v"; tail -5 $OUT/$v.log; exit 1; }
  python3 - $OUT/$v/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith(("void cv::", "cv::")):
        print(f"  {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>3}  {r['Name'][:60]}")
PY
done
