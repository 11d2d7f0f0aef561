set -u
mkdir -p gpurun_out
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/diag/librt_hip_lds_conflicts.so timeout -k 10 300 python scripts/lds_conflicts.py 2 > gpurun_out/lds_conflicts.txt 2>&1; cat gpurun_out/lds_conflicts.txt
rm -f gpurun_out/ab_quick.txt
bash scripts/ab_quick.sh 3 --no-drop-in || exit 1
for l in main shadeglobal ringnoinv; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  for rep in 1 2; do
    timeout -k 10 200 python scripts/rank_emulation.py 1 8 > gpurun_out/emu_${l}_$rep.txt 2>&1 || exit 1
    echo "== $l $rep"; tail -3 gpurun_out/emu_${l}_$rep.txt
  done
done
unset RT_HIP_LIB
for mb in 4 3; do
  RT_EMU_TUNE=max_blocks=$mb timeout -k 10 200 python scripts/rank_emulation.py 1 8 > gpurun_out/emu_mb$mb.txt 2>&1 || exit 1
  echo "== max_blocks $mb"; tail -3 gpurun_out/emu_mb$mb.txt
done
for rep in 1 2 3; do
  for l in main goct_plain; do
    if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
    timeout -k 10 150 python bench.py --scene bunny --no-cpu-baseline --no-drop-in --steps 5 > gpurun_out/bunny_$l.json || exit 1
    python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/bunny_$l.json') if l.startswith('{')][-1])
print('bunny $l', d['ms_per_frame'], d['roofline']['launch_ms'])"
  done
done
for l in main goct_plain; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d gpurun_out/wr_$l -o run -- python bench.py --scene bunny --steps 1 --warmup 0 --no-cpu-baseline --no-drop-in > /dev/null 2>&1 || exit 1
  python3 -c "
import csv, glob
from collections import defaultdict
acc = defaultdict(float)
for f in glob.glob('gpurun_out/wr_$l/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'goct' in r['Kernel_Name']: acc[r['Counter_Name']] += float(r['Counter_Value'])
print('bunny $l render kernel', dict(acc))"
done
