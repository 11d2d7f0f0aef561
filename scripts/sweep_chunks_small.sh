# chunking at smaller launches: 1080p / 512^2 fused and per-frame, 4K per-frame (ms/frame, render ms)
set -u
mkdir -p gpurun_out
out=gpurun_out/sweep_chunks_small.txt; rm -f $out
for rep in 1 2; do
for cfg in "--width 1920 --height 1080" "--width 512 --height 512" "--width 1920 --height 1080 --launch per-frame" \
           "--width 512 --height 512 --launch per-frame" "--launch per-frame"; do
for tn in "chunk_pixels=128 tail_chunk=64" "chunk_pixels=512 tail_chunk=64" "chunk_pixels=512 tail_chunk=128" "chunk_pixels=512 tail_chunk=256"; do
  args=""; for x in $tn; do args="$args --tune $x"; done
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 $cfg $args > gpurun_out/sc.json 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/sc.json') if l.startswith('{')][-1])
print('${cfg}'.replace(' ', '') or 'default', '${tn}'.replace(' ', ','), d['ms_per_frame'], d['roofline']['launch_ms'])" | tee -a $out
done; done; done
