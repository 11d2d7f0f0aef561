"""Ordering of the context's hidden streams against its main stream (csrc/rt_internal.hpp).

The reference has one in-order queue (CLutils.cpp:29); the library keeps that contract while it
runs accumulations, read-backs and gather packs on side streams.  Those side streams wait for the
main stream's tail (main_tail_wait), which is re-recorded only when work may have been enqueued
there since the last record -- so that a record on an idle main stream never lands behind another
stream's packets on a shared hardware queue.  A caller that holds the main stream's handle
(rtContextGetStream) can enqueue there behind the library's back, so from then on the tail is
recorded every time.
"""
import ctypes

import numpy as np
import pytest

from clrt import _native as N


def _hip():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    lib.hipMemsetAsync.restype = ctypes.c_int
    return lib


@pytest.mark.gpu
def test_side_stream_copy_waits_for_work_on_the_exposed_main_stream():
    import clrt
    hip = _hip()
    ctx = clrt.CLContext(0)
    s = ctx.stream()  # the caller now holds the main stream
    ctx.set_readback_on_accum_stream(True)
    n = 1 << 20
    x = ctx.create_buffer(N.MEM_READ_WRITE, n)
    y = ctx.create_buffer(N.MEM_READ_WRITE, n)
    z = ctx.create_buffer(N.MEM_READ_WRITE, 4 << 30)  # ~1 ms of memset ahead of the marker
    ctx.Finish()
    # 1) a side-stream copy: records the main stream's tail
    ctx.CopyRectToDevicePointer(x, 0, n, n, 1, y.device_pointer(), n)
    # 2) the caller writes x on the main stream, behind a long memset, without calling the library
    assert hip.hipMemsetAsync(ctypes.c_void_p(z.device_pointer()), 0, 4 << 30, ctypes.c_void_p(s)) == 0
    assert hip.hipMemsetAsync(ctypes.c_void_p(x.device_pointer()), 0x5A, n, ctypes.c_void_p(s)) == 0
    # 3) the next side-stream copy must see that write (a stale tail would let it run at once)
    ctx.CopyRectToDevicePointer(x, 0, n, n, 1, y.device_pointer(), n)
    ctx.Finish()
    out = np.zeros(n, np.uint8)
    ctx.ReadBuffer(y, out, blocking=True)
    assert (out == 0x5A).all()
    for b in (x, y, z):
        b.release()
    ctx.release()


@pytest.mark.gpu
def test_fused_renders_and_side_copies_after_per_frame_launches(cornell):
    """Per-frame launches write the output on the main stream; a fused render (render stream),
    then a read-back on the accumulation stream, must both come after them -- each mixes a
    main-stream launch with the side streams whose waits skip a clean tail."""
    import clrt
    from hip_helpers import HipRenderer
    W, H = 320, 192
    a = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED)
    b = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED)
    a.ctx.set_readback_on_accum_stream(True)
    dev = a.ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    for f in range(1, 4):  # per-frame, fused, per-frame, fused ...: same bits as all per-frame
        a.frame(f)
        b.frame(f)
    a.frame(4, n_frames=4)
    for f in range(4, 8):
        b.frame(f)
    a.frame(8)
    b.frame(8)
    a.ctx.CopyRectToDevicePointer(a.out, 0, W * 16, W * 16, H, dev.device_pointer(), W * 16)
    a.ctx.Finish()
    got = np.zeros((W * H, 4), np.float32)
    a.ctx.ReadBuffer(dev, got, blocking=True)
    want = b.result()
    assert got[:, :3].tobytes() == want[:, :3].tobytes()
    assert a.result()[:, :3].tobytes() == want[:, :3].tobytes()
    dev.release()
    a.close()
    b.close()
    del clrt
