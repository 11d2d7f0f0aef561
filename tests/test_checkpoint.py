"""GPU: checkpoint / resume of a progressive render.

The reference's render state is its accumulation buffer plus m_FrameCount (CLRaytracer.h:30-37;
KernelEntry reads and rewrites the buffer every frame, kernel_bvh.cl:449-455).  A run stopped after
frame 4, saved (rtiSaveAccum), restored into a NEW context (rtiLoadAccum + WriteBuffer) and taken on
to frame 8 must equal the uninterrupted 8-frame run bit for bit -- through RenderFrame (one launch
per frame) and through fused launches."""
import numpy as np
import pytest

import clrt
from clrt import _native as N
from hip_helpers import HipRenderer

pytestmark = pytest.mark.gpu


def _rt(scene, W, H):
    rt = clrt.Raytracer(W, H)
    rt.Init()
    rt.upload_scene(scene)
    rt.kernel.set_math_mode(N.MATH_SHIPPED)
    return rt


def test_render_frame_checkpoint_resume_equals_uninterrupted(cornell, tmp_path):
    W, H = 320, 180
    ref = _rt(cornell, W, H)
    for _ in range(8):
        ref.RenderFrame()
    want = ref.pixels.copy()
    ref.release()

    a = _rt(cornell, W, H)
    for _ in range(4):
        a.RenderFrame()
    p = str(tmp_path / "run.rtaccum")
    a.checkpoint(p)
    a.release()

    b = _rt(cornell, W, H)
    b.resume(p)
    assert b.frame_count == 5
    for _ in range(4):
        b.RenderFrame()
    assert b.pixels[:, :3].tobytes() == want[:, :3].tobytes()
    b.release()


def test_fused_checkpoint_resume_equals_uninterrupted(cornell, tmp_path):
    from clrt import image
    W, H = 640, 360
    r = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED)
    r.frame(1, n_frames=8)
    want = r.result()
    r.close()

    a = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED)
    a.frame(1, n_frames=4)
    p = str(tmp_path / "fused.rtaccum")
    image.save_accum(p, a.result(), W, H, 5)
    a.close()

    px, nf = image.load_accum(p)
    b = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED)
    b.ctx.WriteBuffer(b.out, px)
    b.frame(nf, n_frames=4)
    assert nf == 5
    assert np.array_equal(b.result()[:, :3].view(np.uint32), want[:, :3].view(np.uint32))
    b.close()
