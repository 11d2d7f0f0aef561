# End-of-session measurement on the final build: GPU tests, smoke, PMC records (profiles/pmc.json
# entries for the default and bunny configs), the default bench with its CPU baseline, a kernel
# trace of the same command, and the other configs.  Everything lands under gpurun_out/final/.
set -u
OUT=gpurun_out/final
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT cmd...
  local n=$1 t=$2; shift 2
  echo "=== $n: $*"
  timeout -k 10 $t "$@" > $OUT/$n.log 2>&1
  local rc=$?
  echo "=== $n rc=$rc"; tail -2 $OUT/$n.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pmc_default 900 bash scripts/profile.sh default
step pmc_bunny 900 bash scripts/profile.sh bunny --scene bunny
cp gpurun_out/pmc_bunny/pmc.json $OUT/pmc.json
cp $OUT/pmc.json profiles/pmc.json
step bench_default 600 python bench.py
step trace_default 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
step bench_bunny 300 python bench.py --scene bunny --no-cpu-baseline
step bench_perframe 300 python bench.py --launch per-frame --no-cpu-baseline --steps 5
step bench_pinned 300 python bench.py --math pinned --no-cpu-baseline --steps 5
step bench_1080p 300 python bench.py --width 1920 --height 1080 --bounces 2 --frames 1 --steps 20 --no-cpu-baseline
step bench_512 300 python bench.py --width 512 --height 512 --bounces 1 --frames 1 --steps 50 --no-cpu-baseline
step bench_bunny_perframe 300 python bench.py --scene bunny --launch per-frame --no-cpu-baseline --steps 3
step bench_wf_cornell 300 python bench.py --sched wavefront --no-cpu-baseline --steps 5
step bench_wf_bunny 300 python bench.py --sched wavefront --scene bunny --no-cpu-baseline --steps 3
step rank_emulation_cornell 400 python scripts/rank_emulation.py
step rank_emulation_bunny 500 env RT_EMU_SCENE=bunny python scripts/rank_emulation.py
step rank_emulation_fused_cornell 400 env RT_EMU_FUSED=1 python scripts/rank_emulation.py
step rank_emulation_fused_bunny 500 env RT_EMU_FUSED=1 RT_EMU_SCENE=bunny python scripts/rank_emulation.py
