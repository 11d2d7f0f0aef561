# Diagnostics of the per-launch tail: build the timeline variant first
# (scripts/build_variant.sh timeline "-DRT_TIMELINE=1"), then run on the GPU box.
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_timeline.so timeout -k 10 200 python scripts/timeline.py 1 8 > gpurun_out/tl.txt 2>&1 || exit 1
for b in 1 3 9; do echo "bounces $b" >> gpurun_out/iso.txt; RT_EMU_ISO=1 RT_EMU_BOUNCES=$b timeout -k 10 200 python scripts/n8_probe.py 1 8 32 >> gpurun_out/iso.txt 2>&1 || exit 1; done
cat gpurun_out/tl.txt gpurun_out/iso.txt
