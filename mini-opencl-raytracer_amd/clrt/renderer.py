"""CLRaytracer without the GL/ImGui half (/root/reference/CLRaytracer.h:14-40).

Init -> SetupBuffers -> (scene upload = CLBVHScene::SetupBuffers) -> RenderFrame, with
the reference's defaults: m_FrameCount starts at 1, lightBounces 9, lightType 0,
skyboxIntensity 1.0 (CLRaytracer.h:30-34) and the CLCamera defaults
(CLcamera.h:8-10).  RenderFrame sets the per-frame uniforms (CLRaytracer.cpp:35-47),
executes W*H work-items, reads the output back and finishes (:51-56), then increments
the frame counter (:101).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import _native as N
from .device import Buffer, CLContext, CLKernel
from .scene import Scene


@dataclass
class Camera:
    """CLCamera defaults (CLcamera.h:8-10)."""
    position: tuple = (0.0, -25.0, 8.5)
    front: tuple = (0.0, 1.0, 0.0)
    up: tuple = (0.0, 0.0, 1.0)


@dataclass
class Raytracer:
    width: int
    height: int
    device: int = 0
    frame_count: int = 1          # m_FrameCount
    light_type: int = 0           # lightType
    light_bounces: int = 9        # lightBounces
    skybox_intensity: float = 1.0  # skyboxIntensity
    frame_seed: int = 0           # rand() in the reference; unused by the kernel
    camera: Camera = field(default_factory=Camera)
    read_back: bool = True        # RenderFrame reads the image back every frame

    def __post_init__(self):
        self.ctx: CLContext | None = None
        self.kernel: CLKernel | None = None
        self.output: Buffer | None = None
        self.pixels = np.zeros((self.height * self.width, 4), np.float32)
        self._scene_bufs: list = []

    # CLRaytracer::Init (CLRaytracer.cpp:104-120)
    def Init(self) -> None:
        self.ctx = CLContext(self.device)
        self.kernel = CLKernel(self.ctx, "KernelEntry")
        self.SetupBuffers()

    # CLRaytracer::SetupBuffers (CLRaytracer.cpp:122-137)
    def SetupBuffers(self) -> None:
        k = self.kernel
        k.set_int(N.WIDTH, self.width)
        k.set_int(N.HEIGHT, self.height)
        self.output = self.ctx.create_buffer(N.MEM_WRITE_ONLY, self.width * self.height * 16)
        k.set_buffer(N.BUFFER_OUT, self.output)

    # CLBVHScene::SetupBuffers (CLBVHnode.cpp:209-236)
    def upload_scene(self, scene: Scene) -> None:
        flags = N.MEM_READ_ONLY | N.MEM_COPY_HOST_PTR
        tb = self.ctx.create_buffer(flags, scene.triangles.nbytes, scene.triangles)
        nb = self.ctx.create_buffer(flags, scene.nodes.nbytes, scene.nodes)
        mb = self.ctx.create_buffer(flags, scene.materials.nbytes, scene.materials)
        for old in self._scene_bufs:
            old.release()
        self._scene_bufs = [tb, nb, mb]
        self.kernel.set_buffer(N.BUFFER_SCENE, tb)
        self.kernel.set_buffer(N.BUFFER_NODE, nb)
        self.kernel.set_buffer(N.BUFFER_MATERIAL, mb)

    def set_uniforms(self) -> None:
        """CLRaytracer::RenderFrame uniform block (CLRaytracer.cpp:35-47)."""
        k = self.kernel
        k.set_uint(N.FRAME_COUNT, self.frame_count)
        k.set_uint(N.FRAME_SEED, self.frame_seed)
        k.set_int(N.LIGHT_BOUNCES, self.light_bounces)
        k.set_int(N.LIGHT_TYPE, self.light_type)
        k.set_float(N.SKYBOX_INTENSITY, self.skybox_intensity)
        k.set_float3(N.CAMERA_POS, self.camera.position)
        k.set_float3(N.CAMERA_FRONT, self.camera.front)
        k.set_float3(N.CAMERA_UP, self.camera.up)

    # CLRaytracer::RenderFrame (CLRaytracer.cpp:12-102), display half removed
    def RenderFrame(self) -> None:
        self.set_uniforms()
        work = self.width * self.height
        self.ctx.ExecuteKernel(self.kernel, work)
        if self.read_back:
            self.ctx.ReadBuffer(self.output, self.pixels, 16 * work)
        self.ctx.Finish()
        self.frame_count += 1

    def image(self) -> np.ndarray:
        """Last read-back frame as (H, W, 3); row 0 is the bottom row (GL order)."""
        return self.pixels.reshape(self.height, self.width, 4)[:, :, :3]

    def save(self, path: str) -> None:
        """Write the last read-back frame (.png, else binary .ppm) -- the display step the
        reference does with glTexSubImage2D (CLRaytracer.cpp:64-67)."""
        from . import image
        w = image.write_png if path.lower().endswith(".png") else image.write_ppm
        w(path, self.pixels, self.width, self.height)

    def checkpoint(self, path: str) -> None:
        """Save the render state -- the accumulation buffer and m_FrameCount (include/rt_image.h
        rtiSaveAccum) -- so a progressive render can resume later from the same bits."""
        from . import image
        px = np.empty((self.height * self.width, 4), np.float32)
        self.ctx.ReadBuffer(self.output, px, blocking=True)
        image.save_accum(path, px, self.width, self.height, self.frame_count)

    def resume(self, path: str) -> None:
        """Restore a checkpoint into this (initialised) raytracer: the next RenderFrame continues
        the accumulation exactly where the saved run stopped."""
        from . import image
        px, nf = image.load_accum(path)
        if px.shape[0] != self.width * self.height:
            raise ValueError("checkpoint size differs from this raytracer's")
        self.ctx.WriteBuffer(self.output, px)
        self.pixels[:] = px
        self.frame_count = nf

    def release(self) -> None:
        for b in self._scene_bufs:
            b.release()
        self._scene_bufs = []
        if self.output:
            self.output.release()
        if self.kernel:
            self.kernel.release()
        if self.ctx:
            self.ctx.release()
