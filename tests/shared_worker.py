"""One rank of a shared world (rtCommInitShared) for tests/test_comm_shared.py: renders its
interleaved bands of a fused 8-frame Cornell render for a few pipelined steps, gathers them to the
root over the copy engines (IPC mappings between the processes), checks a reduction, and the root
saves the gathered image.  usage: shared_worker.py DIR NRANKS RANK W H STEPS ROOT"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from clrt import multigpu as mg  # noqa: E402
from hip_helpers import HipRenderer  # noqa: E402


def main():
    d, n, rank, W, H, steps, root = sys.argv[1], *map(int, sys.argv[2:8])
    r = HipRenderer(clrt.scene.cornell(), W, H, math=N.MATH_SHIPPED)
    comm = mg.Comm.init_shared(r.ctx, n, rank, d)
    assert (comm.rank, comm.nranks) == (rank, n)
    comm.shard(r.k)
    dst = r.ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16) if rank == root else None
    for step in range(steps):
        r.frame(1 + 8 * step, n_frames=8)
        mg.Comm.gather_bands([comm], [r.out], W, H, root=root, dst=dst)
    v = mg.Comm.allreduce([comm], [[float(rank), 1.0]], N.COMM_SUM)
    assert v.tolist() == [[n * (n - 1) / 2, float(n)]], v
    assert comm.transport() == (N.COMM_TRANSPORT_COPY_ENGINES, N.COMM_TRANSPORT_COPY_ENGINES_IPC)
    if rank == root:
        img = np.zeros((W * H, 4), np.float32)
        r.ctx.ReadBuffer(dst, img, blocking=True)
        np.save(os.path.join(d, "gathered.npy"), img)
        dst.release()
    mg.Comm.barrier([comm])  # no rank unmaps the root's memory while others still copy
    comm.destroy()
    r.close()
    print(f"rank {rank} ok")


if __name__ == "__main__":
    main()
