#!/bin/bash
# PMC + kernel-trace profile of the default bench config on the GPU box.
# Each rocprofv3 pass is its own bounded step; counters never share a pass with traces.
# usage: scripts/profile.sh [bench args...]
set -u
OUT=gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline $*"
step() { local n=$1; shift; echo "== $n: $*"; timeout -k 10 600 "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/$n.log; exit $rc; }; }
step list rocprofv3 -L
step trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B
step fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p_fetch -o run -- $B
step write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p_write -o run -- $B
step sq1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/p_sq1 -o run -- $B
step sq2 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/p_sq2 -o run -- $B
step sq3 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/p_sq3 -o run -- $B
python scripts/pmc_summary.py $OUT/summary.json $OUT/p_fetch $OUT/p_write $OUT/p_sq1 $OUT/p_sq2 $OUT/p_sq3
cp $OUT/trace/run_kernel_stats.csv $OUT/kernel_stats.csv 2>/dev/null || true
