set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wavefront.py -x -v --timeout 120 --timeout-method thread > gpurun_out/wf_tests.log 2>&1
echo "tests rc=$?"
tail -5 gpurun_out/wf_tests.log
rc=0
for sc in cornell bunny; do
  timeout -k 10 300 python bench.py --sched wavefront --scene $sc --steps 5 --no-cpu-baseline > gpurun_out/wf_bench_$sc.json 2> gpurun_out/wf_bench_$sc.err || { rc=$?; echo "bench $sc rc=$rc"; tail gpurun_out/wf_bench_$sc.err; break; }
  python -c "import json;d=json.load(open('gpurun_out/wf_bench_$sc.json'));print('$sc', d['ms_per_frame'], d['value'], d['roofline']['kernel_ms'])"
done
exit $rc
