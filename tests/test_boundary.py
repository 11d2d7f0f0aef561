"""CPU tests of the drop-in boundary: the C-ABI libraries load and export every symbol
the headers declare (no compute calls -- there is no GPU here)."""
import ctypes
import os
import re

import pytest

import clrt
from clrt import _native as N

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(REPO, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"\b(rt[si]?[A-Z]\w+)\s*\(", txt)) - {"rtGetErrorString"}


def test_hip_library_exports_header_symbols():
    lib = ctypes.CDLL(clrt.HIP_LIB_PATH)
    names = _declared("rt_hip.h")
    assert len(names) >= 20
    for name in names:
        assert hasattr(lib, name), name
    assert set(N.HIP_EXPORTS) == names


def test_scene_library_exports_header_symbols():
    lib = ctypes.CDLL(clrt.SCENE_LIB_PATH)
    names = _declared("rt_scene.h")
    for name in names:
        assert hasattr(lib, name), name
    assert set(N.SCENE_EXPORTS) == names


def test_image_writer_exports_header_symbols():
    from clrt import image
    lib = ctypes.CDLL(clrt.SCENE_LIB_PATH)
    names = _declared("rt_image.h")
    for name in names:
        assert hasattr(lib, name), name
    assert set(image.IMAGE_EXPORTS) == names


def test_build_info_without_gpu():
    assert b"gfx950" in clrt.hip_lib().rtGetBuildInfo()


def test_no_gpu_fails_loudly():
    """Without a GPU the product raises (no silent CPU fallback)."""
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(clrt.RTError) as e:
        clrt.CLContext(0)
    assert e.value.code in (-1, -33)


def test_layout_matches_reference_struct_sizes():
    # CLshared_structs.hpp:13-87 with 16-byte float3 (CLmathlib.hpp:18-54)
    assert clrt.TRIANGLE_DTYPE.itemsize == 256
    assert clrt.TRIANGLE_DTYPE.fields["mtlIndex"][1] == 240
    assert clrt.NODE_DTYPE.itemsize == 48
    assert clrt.NODE_DTYPE.fields["offset"][1] == 32
    assert clrt.NODE_DTYPE.fields["nPrimitives"][1] == 36
    assert clrt.NODE_DTYPE.fields["axis"][1] == 38
    assert clrt.MATERIAL_DTYPE.itemsize == 64
    assert clrt.MATERIAL_DTYPE.fields["roughness"][1] == 52


def test_error_strings_match_cl_names():
    assert clrt.error_string(-52) == "CL_INVALID_KERNEL_ARGS"
    e = clrt.RTError("Failed to enqueue kernel", -63)
    assert str(e) == "Failed to enqueue kernel (CL_INVALID_GLOBAL_WORK_SIZE)"
