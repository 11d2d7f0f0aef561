"""clrt -- Python host for the MI355X BVH raytracer hot path.

Thin mirror of the reference's host objects over the C ABIs:
  * ``scene.load_obj``      CLOBJloader::Load + CLBVHScene::CreateBVHTrees (librt_scene.so)
  * ``device.CLContext`` / ``device.CLKernel``   CLutils.h:116-145 (librt_hip.so)
  * ``renderer.Raytracer``  CLRaytracer minus the GL/ImGui display half
"""
from ._native import (HIP_EXPORTS, HIP_LIB_PATH, MATERIAL_DTYPE, NODE_DTYPE, SCENE_EXPORTS,
                      SCENE_LIB_PATH, TRIANGLE_DTYPE, RTError, error_string, hip_lib, scene_lib)
from .device import Buffer, CLContext, CLKernel
from .renderer import Camera, Raytracer
from .scene import Scene, build_bvh, load_obj

__all__ = [
    "HIP_EXPORTS", "HIP_LIB_PATH", "MATERIAL_DTYPE", "NODE_DTYPE", "SCENE_EXPORTS", "SCENE_LIB_PATH",
    "TRIANGLE_DTYPE", "RTError", "error_string", "hip_lib", "scene_lib", "Buffer", "CLContext",
    "CLKernel", "Camera", "Raytracer", "Scene", "build_bvh", "load_obj",
]
