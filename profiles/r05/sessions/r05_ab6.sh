# round-5 A/B session 6: per-frame launches (the reference's RenderFrame loop, bench --launch per-frame) on the
# round-4 final tree (_r04, git worktree of b85d132 built in place) against HEAD, Cornell and bunny, 3 rounds
set -u
mkdir -p gpurun_out
rm -f gpurun_out/ab6.txt
for rep in 1 2 3; do
  for t in r04 head; do
    for sc in cornell bunny; do
      if [ $t = r04 ]; then d=_r04; else d=.; fi
      (cd $d && timeout -k 10 150 python bench.py --scene $sc --launch per-frame --no-cpu-baseline --no-drop-in --steps 10) > gpurun_out/ab6_${t}_$sc.json || exit 1
      python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/ab6_${t}_$sc.json') if l.startswith('{')][-1])
print('$t $sc per-frame', d['ms_per_frame'], d['roofline'].get('launch_ms'))" | tee -a gpurun_out/ab6.txt
    done
  done
done
