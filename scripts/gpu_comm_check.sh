#!/bin/bash
# GPU session for the gather: the comm tests, then the world-1 flow on both transports (dist_ab.sh).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_comm.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_comm.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_comm.log; [ $rc -eq 0 ] || exit $rc
DIST_LIBS=main DIST_TAG=copy timeout -k 10 400 bash scripts/dist_ab.sh ${1:-2} || exit $?
DIST_LIBS=main DIST_TAG=rccl timeout -k 10 400 bash scripts/dist_ab.sh 1 --transport rccl
