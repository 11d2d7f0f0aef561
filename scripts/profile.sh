#!/bin/bash
# rocprofv3 profile of one bench.py configuration on the GPU box -> profiles/pmc.json entry.
# A kernel-trace pass, then each PMC pass as its own bounded run (counters never share a pass
# with traces; per-block slot limits of MI355X_MICROARCH.md respected).  Every pass runs the
# SAME command, so bench.py's live roofline can price its own launches with these counts.
# usage: scripts/profile.sh NAME [bench args...]   (outputs under gpurun_out/pmc_NAME)
set -u
NAME=$1; shift
OUT=gpurun_out/pmc_$NAME
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-drop-in --no-configs $*"
step() { local n=$1; shift; echo "== $n"; timeout -k 10 300 "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/$n.log; exit $rc; }; }
step trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B
step fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p_fetch -o run -- $B
step write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p_write -o run -- $B
step sq1 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p_sq1 -o run -- $B
step sq2 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $OUT/p_sq2 -o run -- $B
step wrq rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/p_wrq -o run -- $B
step ta rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum --output-format csv -d $OUT/p_ta -o run -- $B
python scripts/pmc_record.py $OUT/trace $OUT/p_fetch $OUT/p_write $OUT/p_sq1 $OUT/p_sq2 $OUT/p_wrq $OUT/p_ta -- --steps 1 --warmup 0 --no-cpu-baseline --no-drop-in --no-configs "$@" > $OUT/record.txt
cp profiles/pmc.json $OUT/pmc.json
tail -3 $OUT/record.txt
