"""CPU tests of the drop-in boundary: the C-ABI libraries load and export every symbol
the headers declare (no compute calls -- there is no GPU here)."""
import ctypes
import os
import re

import numpy as np
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
    if os.path.exists("/dev/kfd"):
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


# ---- host-side BVH validation (rtValidateBVH; every launch runs it first) -------------------
def _leaf(node, first, count):
    node["nPrimitives"] = count
    node["offset"] = first


def _interior(node, second, axis=0):
    node["nPrimitives"] = 0
    node["offset"] = second
    node["axis"] = axis


def test_validate_bvh_accepts_reference_tree(cornell):
    from clrt import _native as N
    assert N.validate_bvh(cornell.nodes, len(cornell.triangles)) == 6  # depth 7 levels: 0..6


def test_validate_bvh_rejects_shared_child():
    """0 -> (1, 3), 1 -> (2, 3): node 3 has two parents; the skip-pointer walk would loop."""
    from clrt import _native as N
    nd = np.zeros(4, N.NODE_DTYPE)
    _interior(nd[0], 3)
    _interior(nd[1], 3)
    _leaf(nd[2], 0, 1)
    _leaf(nd[3], 1, 1)
    with pytest.raises(clrt.RTError) as e:
        N.validate_bvh(nd, 2)
    assert e.value.code == -38


def test_validate_bvh_orphans_and_trailing_records():
    """Inside the tree (the prefix up to the leaf node 0's chain of second children reaches) an
    unreachable node is rejected; records after the tree are never read, by the reference's
    walk from node 0 either, so they are ignored whatever they hold (rtBuildBVH's node buffer
    has 2n-1 records for a tree of `count`)."""
    from clrt import _native as N
    nd = np.zeros(5, N.NODE_DTYPE)
    _interior(nd[0], 3)
    _leaf(nd[1], 0, 1)
    _leaf(nd[2], 1, 1)  # inside the tree [0, 4) but nobody's child
    _leaf(nd[3], 1, 1)
    _interior(nd[4], 99)
    with pytest.raises(clrt.RTError) as e:
        N.validate_bvh(nd, 2)
    assert e.value.code == -38
    nd = np.zeros(6, N.NODE_DTYPE)
    _interior(nd[0], 2)
    _leaf(nd[1], 0, 1)
    _leaf(nd[2], 1, 1)
    _interior(nd[3], 99)  # past the tree: garbage allowed
    _interior(nd[4], 1)
    assert N.validate_bvh(nd, 2) == 1
    nd = np.zeros(3, N.NODE_DTYPE)
    _interior(nd[0], 7)  # the root's second child past the buffer
    with pytest.raises(clrt.RTError):
        N.validate_bvh(nd, 2)


@pytest.mark.parametrize("case", ["cycle", "leaf_range", "axis", "backward"])
def test_validate_bvh_rejects_malformed(cornell, case):
    from clrt import _native as N
    bad = cornell.nodes.copy()
    interior = np.flatnonzero(bad["nPrimitives"] == 0)
    leaf = np.flatnonzero(bad["nPrimitives"] > 0)[0]
    if case == "cycle":
        bad["offset"][interior[0]] = interior[0]
    elif case == "leaf_range":
        bad["offset"][leaf] = len(cornell.triangles) - 1
        bad["nPrimitives"][leaf] = 2
    elif case == "axis":
        bad["axis"][interior[1]] = 3
    else:
        bad["offset"][interior[2]] = interior[2] - 1
    with pytest.raises(clrt.RTError):
        N.validate_bvh(bad, len(cornell.triangles))
