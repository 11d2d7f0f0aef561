"""GPU: bench.py's N > 1 flow -- the launcher's environment (WORLD_SIZE / RANK / LOCAL_RANK /
MASTER_*), the per-launch file rendezvous, sharded fused renders, the pipelined gather every step,
max-over-ranks timing and rank 0's single JSON line -- with 2 ranks on the test box's one GPU as a
shared world (--shared-world: no RCCL, which refuses two ranks on one device; gathers over IPC
mappings on the copy engines).  --check-gather: rank 0 re-renders the frame unsharded and
compares the gathered image byte for byte."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_shared_world(tmp_path):
    world = 2
    base = dict(os.environ, WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(41000 + os.getpid() % 1000), RT_COMM_ID_FILE=str(tmp_path / "comm.id"))
    args = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(world), "--shared-world", "--check-gather",
            "--width", "640", "--height", "360", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    procs = [subprocess.Popen(args, env=dict(base, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=110))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), "\n".join(o[1][-1500:] for o in outs)
    lines = [l for l in outs[0][0].splitlines() if l.startswith("{")]
    assert len(lines) == 1 and not [l for l in outs[1][0].splitlines() if l.startswith("{")]
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["value"] > 0
    assert "byte-identical" in d["check_gather"] and "(2 ranks)" in d["check_gather"]
    assert "shared world" in d["config"]["parallelism"]
