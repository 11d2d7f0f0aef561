#!/bin/bash
# A/B of one experimental build (scripts/build_variant.sh NAME) against the main build on the
# emulated ranks (fused 4K 8 spp, N = 1 and 8, both scenes, two rounds), after the full-size
# benched-path parity tests on the variant.  usage: ab_variant_emu.sh NAME
set -u
V=mini-opencl-raytracer_amd/lib/variants/librt_hip_$1.so
O=gpurun_out/ab_$1
mkdir -p $O
RT_HIP_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_benched_path.py tests/test_fused_frames.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for sc in cornell bunny; do
    for lib in main $1; do
      echo "== $sc lib=$lib" >> $O/ab.txt
      if [ $lib = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$V; fi
      RT_EMU_FUSED=1 RT_EMU_SCENE=$sc timeout -k 10 120 python scripts/rank_emulation.py 1 8 >> $O/ab.txt 2>&1 || exit 1
    done
  done
done
unset RT_HIP_LIB
cat $O/ab.txt
