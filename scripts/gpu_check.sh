#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; the script stops at the first step that
# crashed, aborted or timed out (exit >= 124 or a signal), and continues past plain
# test failures (exit 1) so one call still yields a bench line and a profile.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 $OUT/$name.log
  if [ $rc -ge 124 ] || [ $rc -gt 1 ] && [ $rc -ne 5 ]; then
    echo "stopping after $name (rc=$rc)" | tee -a $OUT/steps.log
    exit $rc
  fi
  return 0
}
(clinfo 2>&1 | head -60 > $OUT/clinfo.txt) || true
(rocm-smi --showproductname 2>&1 | head -20 > $OUT/smi.txt) || true
nproc > $OUT/nproc.txt; (lscpu | head -20 >> $OUT/nproc.txt) || true
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu --maxfail 8 -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs ;;
    dist1) run dist1_rccl 300 python bench.py --force-dist --check-gather --steps 5 --warmup 1 --no-cpu-baseline && \
           run dist1_rccl_sync 300 python bench.py --force-dist --gather-sync --steps 5 --warmup 1 --no-cpu-baseline ;;
    pmc) run pmc_default 900 bash scripts/profile.sh default ;;
    pmcbunny) run pmc_bunny 900 bash scripts/profile.sh bunny --scene bunny ;;
    benchbunny) run bench_bunny 600 python bench.py --scene bunny --no-cpu-baseline --steps 3 ;;
    phase) run phase 300 python scripts/phase_profile.py ;;
    phasebunny) RT_PHASE_SCENE=bunny run phase_bunny 300 python scripts/phase_profile.py ;;
    refgold) run refgold 900 python scripts/make_ref_goldens.py gpurun_out/golden ;;
    # the round's final record (what the round-3 final_r03_{a,b,c,d}.sh did, by step):
    #   final_suite: GPU suite (long per-test limit) + smoke on the final build
    final_suite) run pytest_gpu 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread && \
                 run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    #   final_bench: PMC records (headline + bunny -> profiles/pmc.json), the default bench with its CPU
    #   baseline and drop-in figures, and a kernel trace of the timed loop
    #   (round 6: also the PMC keys of the bench line's other configs -- bench.py EXTRA_CONFIGS)
    final_bench) run pmc_default 900 bash scripts/profile.sh default && \
                 run pmc_bunny 900 bash scripts/profile.sh bunny --scene bunny && \
                 run pmc_1080p 900 bash scripts/profile.sh 1080p --width 1920 --height 1080 --bounces 2 --frames 1 && \
                 run pmc_pinned 900 bash scripts/profile.sh pinned --math pinned && \
                 cp gpurun_out/pmc_pinned/pmc.json profiles/pmc.json && \
                 run bench_default 600 python bench.py && \
                 run bench_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/final_trace -o run -- python bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-drop-in --no-configs ;;
    #   final_configs: the other configs (no CPU baseline / drop-in) and the emulated ranks
    final_configs) for c in "bunny --scene bunny" "perframe --launch per-frame --steps 5" "pinned --math pinned --steps 5" \
                             "1080p --width 1920 --height 1080 --bounces 2 --frames 1 --steps 20" \
                             "512 --width 512 --height 512 --bounces 1 --frames 1 --steps 50" \
                             "bunny_perframe --scene bunny --launch per-frame --steps 3"; do
                     set -- $c; n=$1; shift
                     run bench_$n 300 python bench.py --no-cpu-baseline --no-drop-in --no-configs "$@"
                   done
                   for sc in cornell bunny; do
                     RT_EMU_SCENE=$sc run rank_emulation_$sc 600 python scripts/rank_emulation.py
                   done ;;
    configs) run cfg3_default 600 python bench.py && \
             run cfg3_pinned 300 python bench.py --math pinned --no-cpu-baseline && \
             run cfg2_1080p 300 python bench.py --width 1920 --height 1080 --bounces 2 --frames 1 --steps 20 --no-cpu-baseline && \
             run cfg1_512 300 python bench.py --width 512 --height 512 --bounces 1 --frames 1 --steps 50 --no-cpu-baseline && \
             run cfg5_bunny 300 python bench.py --scene bunny --no-cpu-baseline && \
             run cfg5_bunny_pinned 300 python bench.py --scene bunny --math pinned --no-cpu-baseline ;;
    *) echo "unknown step $step" ;;
  esac
done
