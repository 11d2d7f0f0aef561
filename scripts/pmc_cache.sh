# L1/L2 cache counters of one bench command (per kernel, summed): scripts/pmc_sum.py gpurun_out/pmcc_NAME
set -u
NAME=$1; shift
OUT=gpurun_out/pmcc_$NAME
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline $*"
step() { local n=$1; shift; timeout -k 10 300 "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/$n.log; exit $rc; }; }
step trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B
step tcc rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/p_tcc -o run -- $B
step tcp rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d $OUT/p_tcp -o run -- $B
step sq rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU --output-format csv -d $OUT/p_sq -o run -- $B
