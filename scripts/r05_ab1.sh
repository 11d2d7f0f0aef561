set -u
mkdir -p gpurun_out
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/diag/librt_hip_lds_conflicts.so timeout -k 10 300 python scripts/lds_conflicts.py 2 > gpurun_out/lds_conflicts.txt 2>&1; cat gpurun_out/lds_conflicts.txt
rm -f gpurun_out/ab_quick.txt
bash scripts/ab_quick.sh 3 --no-drop-in || exit 1
for l in main shadeglobal; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  for rep in 1 2; do
    timeout -k 10 200 python scripts/rank_emulation.py 1 8 > gpurun_out/emu_${l}_$rep.txt 2>&1 || exit 1
    echo "== $l $rep"; tail -3 gpurun_out/emu_${l}_$rep.txt
  done
done
