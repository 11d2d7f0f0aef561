# PMC passes of one bench command, summed per kernel over its dispatches (scripts/pmc_sum.py)
# usage: scripts/pmc_kernels.sh NAME [bench args...]
set -u
NAME=$1; shift
OUT=gpurun_out/pmck_$NAME
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline $*"
step() { local n=$1; shift; timeout -k 10 300 "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/$n.log; exit $rc; }; }
step trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B
step sq1 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p_sq1 -o run -- $B
step sq2 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/p_sq2 -o run -- $B
step fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p_fetch -o run -- $B
step write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p_write -o run -- $B
