#!/bin/bash
# emulated 8-rank step (max over ranks) under work-distribution knobs: scripts/sweep_emu8.sh SCENE
set -u
for e in "RT_NONE=1" "RT_BULK_PERCENT=60" "RT_BULK_PERCENT=90" "RT_CHUNK=64" "RT_CHUNK=256" "RT_TAIL_CHUNK=128"; do
  out=$(env $e RT_EMU_SCENE=$1 RT_EMU_FUSED=1 RT_EMU_STEPS=3 timeout -k 10 120 python scripts/rank_emulation.py 8 | grep "^N=8") || exit $?
  echo "$1 [$e] $(echo $out | sed 's/.*| max \([0-9.]*\) |.*/max \1/')"
done
