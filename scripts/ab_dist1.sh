#!/bin/bash
# A/B of the pipelined gather's pack stream at world size 1 over RCCL, alternating, 20 steps.
set -u
port=29540
for rep in 1 2 3; do
  for ps in main accum; do
    port=$((port + 1))
    out=$(timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
          --master-port $port bench.py --force-dist --no-cpu-baseline --pack-stream $ps 2>/dev/null | grep '^{') || exit $?
    echo "$ps $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"])')"
  done
done
