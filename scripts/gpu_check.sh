#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; the script stops at the first step that
# crashed, aborted or timed out (exit >= 124 or a signal), and continues past plain
# test failures (exit 1) so one call still yields a bench line and a profile.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 $OUT/$name.log
  if [ $rc -ge 124 ] || [ $rc -gt 1 ] && [ $rc -ne 5 ]; then
    echo "stopping after $name (rc=$rc)" | tee -a $OUT/steps.log
    exit $rc
  fi
  return 0
}
(clinfo 2>&1 | head -60 > $OUT/clinfo.txt) || true
(rocm-smi --showproductname 2>&1 | head -20 > $OUT/smi.txt) || true
nproc > $OUT/nproc.txt; (lscpu | head -20 >> $OUT/nproc.txt) || true
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 900 python -m pytest tests -m gpu -x -q ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    benchdl) run bench_devicelib 600 python bench.py --math devicelib --no-cpu-baseline ;;
    benchstep) run bench_pin_step 600 python bench.py --sched step --no-cpu-baseline && \
             run bench_dl_step 600 python bench.py --math devicelib --sched step --no-cpu-baseline && \
             run bench_dl_regen 600 python bench.py --math devicelib --sched regen --no-cpu-baseline ;;
    benchab) run bench_pin_tiles 600 python bench.py --sched tiles --no-cpu-baseline && \
             run bench_pin_regen 600 python bench.py --sched regen --no-cpu-baseline && \
             run bench_dl_tiles 600 python bench.py --math devicelib --sched tiles --no-cpu-baseline && \
             run bench_dl_regen 600 python bench.py --math devicelib --sched regen --no-cpu-baseline ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    dist2) run dist2_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --math devicelib ;;
    dist1) run dist1_nccl_pipelined 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --force-dist --check-gather --steps 5 --warmup 1 --no-cpu-baseline && \
           run dist1_nccl_sync 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29535 bench.py --force-dist --no-overlap --steps 5 --warmup 1 --no-cpu-baseline ;;
    benchbunny) run bench_bunny 600 python bench.py --scene bunny --no-cpu-baseline --steps 3 ;;
    phase) run phase 300 python scripts/phase_profile.py ;;
    phasebunny) RT_PHASE_SCENE=bunny run phase_bunny 300 python scripts/phase_profile.py ;;
    pmcbunny) run pmcb_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcb_fetch -o run -- python bench.py --scene bunny --steps 1 --warmup 0 --no-cpu-baseline && \
              run pmcb_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmcb_sq -o run -- python bench.py --scene bunny --steps 1 --warmup 0 --no-cpu-baseline && \
              run pmcb_sq2 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmcb_sq2 -o run -- python bench.py --scene bunny --steps 1 --warmup 0 --no-cpu-baseline && \
              python scripts/pmc_summary.py $OUT/pmcb_summary.json $OUT/pmcb_fetch $OUT/pmcb_sq $OUT/pmcb_sq2 > $OUT/pmcb_summary.txt ;;
    phasepool) run phase_pool 300 python scripts/phase_profile.py step pool ;;
    poolpar) run pool_parity 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "schedules or interleaved" ;;
    benchpool) run bench_pool_dl 600 python bench.py --sched pool --no-cpu-baseline && \
               run bench_pool_pin 600 python bench.py --sched pool --math pinned --no-cpu-baseline ;;
    refgold) run refgold 900 python scripts/make_ref_goldens.py gpurun_out/golden ;;
    pmc) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline && \
         run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline ;;
    variants) for m in devicelib pinned; do \
                for v in mini-opencl-raytracer_amd/lib/variants/*.so; do n=$(basename $v .so); \
                  RT_HIP_LIB=$v run ab_${n}_$m 300 python bench.py --math $m --no-cpu-baseline --steps 3 || exit $?; done; \
                run ab_main_$m 300 python bench.py --math $m --no-cpu-baseline --steps 3 || exit $?; done ;;
    configs) run cfg3_default 600 python bench.py && \
             run cfg3_pinned 300 python bench.py --math pinned --no-cpu-baseline && \
             run cfg2_1080p 300 python bench.py --width 1920 --height 1080 --bounces 2 --frames 1 --steps 20 --no-cpu-baseline && \
             run cfg1_512 300 python bench.py --width 512 --height 512 --bounces 1 --frames 1 --steps 50 --no-cpu-baseline && \
             run cfg5_bunny 300 python bench.py --scene bunny --no-cpu-baseline && \
             run cfg5_bunny_pinned 300 python bench.py --scene bunny --math pinned --no-cpu-baseline ;;
    *) echo "unknown step $step" ;;
  esac
done
