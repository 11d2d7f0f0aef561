#!/bin/bash
# bench.py's N > 1 flow with N ranks sharing the box's one GPU as a shared world (--shared-world:
# no RCCL; gathers over IPC mappings on the copy engines), launched like torch.distributed.run
# would (WORLD_SIZE / RANK / LOCAL_RANK / MASTER_*), without importing torch.  Not a scaling
# measurement: the ranks share one GPU, so the aggregate shows what the N-rank flow costs on it.
# usage: scripts/shared_bench.sh N [bench args...]   (rank 0's JSON line on stdout)
set -u
N=$1; shift
mkdir -p gpurun_out
export WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=$((42000 + $$ % 1000))
export RT_COMM_ID_FILE=/tmp/rt_shared_bench_$$.id
pids=()
for r in $(seq 0 $((N - 1))); do
  RANK=$r LOCAL_RANK=$r timeout -k 10 300 python bench.py --gpus $N --shared-world "$@" > gpurun_out/shared_bench_r$r.out 2> gpurun_out/shared_bench_r$r.err &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
rm -f $RT_COMM_ID_FILE
[ $rc -eq 0 ] || { tail -5 gpurun_out/shared_bench_r*.err; exit $rc; }
grep "^{" gpurun_out/shared_bench_r0.out
