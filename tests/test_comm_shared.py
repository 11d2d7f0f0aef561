"""GPU: a world of separate processes on the one GPU of the test box (rtCommInitShared: setup
through files, no RCCL, which refuses two ranks on one device).  The gathers then take the path
the one-process-per-GPU setup takes between GPUs -- IPC handles of the root's receive slots and
flags exchanged and mapped, the link handshake, copy-engine copies into another process's memory,
arrival and slot-free flags written into another process's memory and waited on -- over several
pipelined steps (slots reused); only the copy between two GPUs over xGMI is not exercised.  The
gathered image must be byte-identical to an unsharded render."""
import os
import subprocess
import sys

import numpy as np
import pytest

from clrt import _native as N
from hip_helpers import HipRenderer

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("n,root,W,H", [(2, 0, 640, 360), (3, 1, 517, 203)])
def test_shared_world_gather_equals_unsharded(cornell, tmp_path, n, root, W, H):
    steps = 4
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "shared_worker.py"), str(tmp_path), str(n),
                               str(q), str(W), str(H), str(steps), str(root)],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for q in range(n)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=100)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), "\n".join(o[-1500:] for o in outs)
    got = np.load(tmp_path / "gathered.npy")
    r = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED)
    for step in range(steps):
        r.frame(1 + 8 * step, n_frames=8)
    want = r.result()
    r.close()
    assert got.tobytes() == want.tobytes(), f"{(got != want).any(axis=1).sum()} pixels differ"


def test_shared_world_refuses_rccl_and_bad_arguments(tmp_path):
    import clrt
    from clrt import multigpu as mg
    ctx = clrt.CLContext(0)
    with pytest.raises(Exception):
        mg.Comm.init_shared(ctx, 2, 2, str(tmp_path))
    comm = mg.Comm.init_shared(ctx, 1, 0, str(tmp_path))
    with pytest.raises(Exception):
        comm.set_transport(N.COMM_TRANSPORT_RCCL)
    comm.set_transport(N.COMM_TRANSPORT_COPY_ENGINES)
    mg.Comm.barrier([comm])
    comm.destroy()
    # the directory now holds that world's id: a new world there is refused (its exchange files
    # could be read as the new world's)
    with pytest.raises(Exception) as e:
        mg.Comm.init_shared(ctx, 1, 0, str(tmp_path))
    assert e.value.code == -30
    ctx.release()
