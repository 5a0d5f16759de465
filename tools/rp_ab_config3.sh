set -u
mkdir -p gpurun_out/ab2
export TMPDIR=/tmp
for L in - cilium_amd/_lib/ab/lib_4ab12b3.so; do
  n=$(basename "$L" .so); if [ "$L" = "-" ]; then n=head; unset CV_LIB; else export CV_LIB=$PWD/$L; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab2/$n -o run --output-format csv -- python3 bench.py --workload config3 --steps 6 --warmup 1 --no-cpu > gpurun_out/ab2/$n.log 2>&1 || exit 1
done
