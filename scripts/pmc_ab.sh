#!/bin/bash
# SQ counter passes for several schedules (A/B of the step and pool schedules).
# usage: scripts/pmc_ab.sh sched [sched ...]
set -u
export TMPDIR=/tmp
for s in "$@"; do
  OUT=gpurun_out/pmc_$s
  mkdir -p $OUT
  B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --sched $s"
  step() { local n=$1; shift; echo "== $s $n"; timeout -k 10 300 "$@" > $OUT/$n.log 2>&1; local rc=$?; [ $rc -eq 0 ] || { tail -20 $OUT/$n.log; exit $rc; }; }
  step sq1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/p_sq1 -o run -- $B
  step sq2 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/p_sq2 -o run -- $B
  step sq3 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/p_sq3 -o run -- $B
  python scripts/pmc_summary.py $OUT/summary.json $OUT/p_sq1 $OUT/p_sq2 $OUT/p_sq3 > $OUT/summary.txt
done
