# Rehearsal of the N=2 bench flow with both ranks on the box's one GPU (RCCL permitting):
# WORLD_SIZE=2, LOCAL_RANK=0 for both, rendezvous through RT_COMM_ID_FILE.
set -u
mkdir -p gpurun_out
export NCCL_DEBUG=WARN RT_COMM_ID_FILE=/tmp/rt_two_ranks.id WORLD_SIZE=2 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
rm -f $RT_COMM_ID_FILE
A="--width 1280 --height 720 --steps 3 --warmup 1 --no-cpu-baseline --check-gather --gpus 2"
RANK=1 timeout -k 10 120 python bench.py $A > gpurun_out/two_r1.log 2>&1 &
p1=$!
RANK=0 timeout -k 10 120 python bench.py $A > gpurun_out/two_r0.log 2>&1
r0=$?
wait $p1; r1=$?
echo "rank0 rc=$r0 rank1 rc=$r1"
tail -3 gpurun_out/two_r0.log; tail -3 gpurun_out/two_r1.log
