#!/bin/bash
# GPU session for the gather: the comm / stream-order / coalescing tests, then the world-1 flow
# (dist_ab.sh: the bench with and without the gather every step) on each transport.
# usage: scripts/gpu_comm_check.sh [REPS] [TRANSPORTS...]   (default: 2 copy-ipc copy rccl)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
reps=${1:-2}; shift || true
transports=${*:-"copy-ipc copy rccl"}
timeout -k 10 900 python -u -m pytest tests/test_comm.py tests/test_comm_shared.py tests/test_bench_shared.py \
  tests/test_frame_coalescing.py tests/test_stream_order.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_comm.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_comm.log; [ $rc -eq 0 ] || exit $rc
for t in $transports; do
  DIST_LIBS=main DIST_TAG=$t timeout -k 10 500 bash scripts/dist_ab.sh $reps --transport $t || exit $?
done
