"""Drive librt_hip.so the way the reference's RenderFrame drives its OpenCL kernel."""
import numpy as np

import clrt
from clrt import _native as N

DEFAULT_CAMERA = ((0.0, -25.0, 8.5), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0))


def _cross32(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]],
                    np.float32)


def reference_camera(pitch=None, yaw=None, moves=()):
    """The camera the reference's UI hands to KernelEntry (slots 11-13, CLRaytracer.cpp:42-47).

    Starts from CLCamera's defaults (CLcamera.h:8-13).  A (pitch, yaw) drag runs
    CLCamera::Update (CLcamera.h:15-21; CLui.cpp:221-228): front = (cos yaw sin pitch,
    sin yaw sin pitch, cos pitch) in fp32, up unchanged.  `moves` are arrow keys in order
    (CLEngineBase.cpp:141-162): "up" pos += front, "down" pos -= front, "right"
    pos += cross(front, up), "left" pos -= cross(front, up).  Returns (pos, front, up) as
    Python floats of the fp32 values."""
    pos = np.array([0.0, -25.0, 8.5], np.float32)
    front = np.array([0.0, 1.0, 0.0], np.float32)
    up = np.array([0.0, 0.0, 1.0], np.float32)
    if pitch is not None:
        p, y = np.float32(pitch), np.float32(yaw)
        front = np.array([np.cos(y) * np.sin(p), np.sin(y) * np.sin(p), np.cos(p)], np.float32)
    for m in moves:
        if m == "up":
            pos = pos + front
        elif m == "down":
            pos = pos - front
        elif m == "right":
            pos = pos + _cross32(front, up)
        elif m == "left":
            pos = pos - _cross32(front, up)
        else:
            raise ValueError(m)
    return tuple(tuple(float(c) for c in v) for v in (pos, front, up))


class HipRenderer:
    """One context + kernel + scene + output buffer; frames rendered on demand."""

    def __init__(self, scene, width, height, math=N.MATH_PINNED, device=0, hits=False,
                 stats=False, force_global=False, global_size=None, sched=N.SCHED_STEP, perframe_batch=1):
        self.W, self.H = width, height
        self.n = global_size if global_size is not None else width * height
        self.ctx = clrt.CLContext(device)
        self.k = clrt.CLKernel(self.ctx, "KernelEntry")
        flags = N.MEM_READ_ONLY | N.MEM_COPY_HOST_PTR
        self.bufs = [self.ctx.create_buffer(flags, a.nbytes, a)
                     for a in (scene.triangles, scene.nodes, scene.materials)]
        self.out = self.ctx.create_buffer(N.MEM_WRITE_ONLY, max(self.n, width * height) * 16)
        self.k.set_buffer(N.BUFFER_OUT, self.out)
        self.k.set_buffer(N.BUFFER_SCENE, self.bufs[0])
        self.k.set_buffer(N.BUFFER_NODE, self.bufs[1])
        self.k.set_buffer(N.BUFFER_MATERIAL, self.bufs[2])
        self.k.set_int(N.WIDTH, width)
        self.k.set_int(N.HEIGHT, height)
        self.k.set_math_mode(math)
        self.k.set_schedule(sched)
        self.k.force_global_scene(force_global)
        self.k.set_stats(stats)
        # per-frame launches launch one by one (the per-frame baselines the tests compare against);
        # frame coalescing is the subject only where a test asks for it (perframe_batch > 1, or
        # None: the library default)
        if perframe_batch is not None:
            self.k.set_tuning("perframe_batch", perframe_batch)
        self.hit_bufs = None
        if hits:
            self.hit_bufs = (self.ctx.create_buffer(N.MEM_READ_WRITE, self.n * 4),
                             self.ctx.create_buffer(N.MEM_READ_WRITE, self.n * 4))
            self.k.set_hit_buffers(*self.hit_bufs)

    def frame(self, frame_count, light_bounces=9, light_type=0, skybox=1.0, camera=DEFAULT_CAMERA,
              work_range=None, interleave=None, n_frames=None):
        """One KernelEntry launch (RenderFrame), or with n_frames: frames frame_count ..
        frame_count + n_frames - 1 through rtEnqueueKernelFrames."""
        k = self.k
        k.set_uint(N.FRAME_COUNT, frame_count)
        k.set_uint(N.FRAME_SEED, 12345)
        k.set_int(N.LIGHT_BOUNCES, light_bounces)
        k.set_int(N.LIGHT_TYPE, light_type)
        k.set_float(N.SKYBOX_INTENSITY, skybox)
        k.set_float3(N.CAMERA_POS, camera[0])
        k.set_float3(N.CAMERA_FRONT, camera[1])
        k.set_float3(N.CAMERA_UP, camera[2])
        if work_range is not None:
            k.set_work_range(*work_range)
        if interleave is not None:
            k.set_row_interleave(*interleave)
        if n_frames is None:
            self.ctx.ExecuteKernel(k, self.n)
        else:
            self.ctx.ExecuteKernelFrames(k, self.n, n_frames)

    def result(self):
        out = np.zeros((self.n, 4), np.float32)
        self.ctx.ReadBuffer(self.out, out, self.n * 16, blocking=True)
        return out

    def hits(self):
        ids = np.zeros(self.n, np.int32)
        t = np.zeros(self.n, np.float32)
        self.ctx.ReadBuffer(self.hit_bufs[0], ids, blocking=True)
        self.ctx.ReadBuffer(self.hit_bufs[1], t, blocking=True)
        return ids, t

    def close(self):
        self.ctx.Finish()
        if self.hit_bufs:
            for b in self.hit_bufs:
                b.release()
        for b in self.bufs:
            b.release()
        self.out.release()
        self.k.release()
        self.ctx.release()


def rgb(a):
    return np.ascontiguousarray(a[:, :3])
