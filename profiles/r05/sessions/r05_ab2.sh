# round-5 A/B session 2: the round-4 final tree (_r04, git worktree of b85d132, built in place) against
# HEAD on both headline configs, then the tail-shading / tail-priority variants (default bench and the
# emulated N=8 rank).
set -u
mkdir -p gpurun_out
rm -f gpurun_out/ab_r04.txt gpurun_out/ab_quick.txt
for rep in 1 2 3; do
  for t in r04 head; do
    for sc in cornell bunny; do
      if [ $t = r04 ]; then d=_r04; else d=.; fi
      (cd $d && timeout -k 10 150 python bench.py --scene $sc --no-cpu-baseline --no-drop-in --steps 10) > gpurun_out/ab_${t}_$sc.json || exit 1
      python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/ab_${t}_$sc.json') if l.startswith('{')][-1])
print('$t $sc', d['ms_per_frame'], d['roofline'].get('launch_ms', d['roofline'].get('kernel_ms')))" | tee -a gpurun_out/ab_r04.txt
    done
  done
done
bash scripts/ab_quick.sh 3 --no-drop-in || exit 1
for l in main tailshade2 tailshade8 tailprio; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  timeout -k 10 200 python scripts/rank_emulation.py 1 8 > gpurun_out/emu2_$l.txt 2>&1 || exit 1
  echo "== $l"; tail -2 gpurun_out/emu2_$l.txt
done
