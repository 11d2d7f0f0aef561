# final round-3 measurement, part C: the other configs and the emulated multi-GPU rank steps
set -o pipefail
OUT=gpurun_out/final_r03; mkdir -p $OUT; export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-drop-in "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || exit 1; }
b bunny --scene bunny
b perframe --launch per-frame --steps 5
b pinned --math pinned --steps 5
b 1080p --width 1920 --height 1080 --bounces 2 --frames 1 --steps 20
b 512 --width 512 --height 512 --bounces 1 --frames 1 --steps 50
b bunny_perframe --scene bunny --launch per-frame --steps 3
for sc in cornell bunny; do
  RT_EMU_FUSED=1 RT_EMU_SCENE=$sc timeout -k 10 500 python scripts/rank_emulation.py > $OUT/rank_emulation_fused_$sc.txt 2>&1 || exit 1
done
