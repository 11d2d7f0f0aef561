# final round-3 measurement, part B: PMC records of the headline and the bunny proxy, the default
# bench (with its CPU baseline and the drop-in figures) and a rocprofv3 kernel trace of it
set -o pipefail
OUT=gpurun_out/final_r03; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/profile.sh default || exit 1
bash scripts/profile.sh bunny --scene bunny || exit 1
cp gpurun_out/pmc_bunny/pmc.json profiles/pmc.json
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-drop-in > $OUT/trace.log 2>&1 || exit 1
