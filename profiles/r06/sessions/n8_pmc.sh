#!/bin/bash
# Round 6 diagnostic: VALU issue of the emulated N = 8 rank loop (rank 3's bands, fused, 10 steps) against N = 1:
# kernel trace + one SQ counter pass of each (scripts/rank_emulation.py with one N per run).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/n8pmc
for n in 1 8; do
  RT_EMU_FUSED=1 RT_EMU_SCENE=cornell RT_EMU_STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/n8pmc/trace_$n -o run -- python3 scripts/rank_emulation.py $n > gpurun_out/n8pmc/trace_$n.log 2>&1 || exit 1
  RT_EMU_FUSED=1 RT_EMU_SCENE=cornell RT_EMU_STEPS=10 timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/n8pmc/pmc_$n -o run -- python3 scripts/rank_emulation.py $n > gpurun_out/n8pmc/pmc_$n.log 2>&1 || exit 1
done
