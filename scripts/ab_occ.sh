set -u
mkdir -p gpurun_out/occ
for v in dw4 dw5 main; do
  if [ $v = main ]; then L=""; else L="RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$v.so"; fi
  env $L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/occ/bench_$v.log 2>&1 || exit $?
  env $L timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/occ/w_$v -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/occ/pw_$v.log 2>&1 || exit $?
done
