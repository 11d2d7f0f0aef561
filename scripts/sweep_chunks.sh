# work-counter chunking of the fused step render (bulk chunk pixels, tail chunk, bulk share),
# ms/frame and render ms; SCENE=bunny for the HBM/L2 path, LAUNCH=per-frame, EXTRA=bench args
set -u
mkdir -p gpurun_out
out=gpurun_out/sweep_chunks_${SCENE:-cornell}${TAG:-}.txt; rm -f $out
for rep in 1 2; do
for c in ${CHUNKS:-512 1024 2048}; do for t in ${TAILS:-256 512 1024}; do for b in ${BULKS:-80 90 100}; do
  tn="chunk_pixels=$c tail_chunk=$t bulk_percent=$b"
  args=""; for x in $tn; do args="$args --tune $x"; done
  timeout -k 10 120 python bench.py --scene ${SCENE:-cornell} --launch ${LAUNCH:-fused} --no-cpu-baseline --steps 10 $args ${EXTRA:-} > gpurun_out/sc.json 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/sc.json') if l.startswith('{')][-1])
print('${tn}'.replace(' ', ','), d['ms_per_frame'], d['roofline']['launch_ms'])" | tee -a $out
done; done; done
done
