# kernel trace of the wavefront schedule (per-kernel, per-bounce durations)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for sc in ${SCENES:-cornell bunny}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wfprof_$sc -o run -- python bench.py --sched wavefront --scene $sc --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/wfprof_$sc.log 2>&1 || { echo "prof $sc failed"; tail gpurun_out/wfprof_$sc.log; exit 1; }
done
