# final round-3 measurement, part D: GPU suite + smoke on the last build, and the bunny proxy lines it changed
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/final_r03; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-drop-in --scene bunny > $OUT/bench_bunny.json 2> $OUT/bench_bunny.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-drop-in --scene bunny --launch per-frame --steps 3 > $OUT/bench_bunny_perframe.json 2> $OUT/bench_bunny_perframe.err || exit 1
grep '^{' $OUT/bench_bunny.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bunny', d['ms_per_frame'], d['value'], d['roofline'].get('frac'), d['roofline'].get('ta_busy'))"
