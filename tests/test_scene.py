"""CPU: the host scene pipeline (librt_scene.so) -- the OBJ/MTL loader restating
CLOBJloader.cpp:10-176 and the SAH BVH build/flatten restating CLBVHnode.cpp:7-207.

Pinned by: the SURVEY's probe of the reference host compiled in place (Cornell: 72
triangles, 6 materials, 39 nodes, 20 leaves, <= 4 primitives per leaf, depth 7), the
probe counts tests/test_oracle.py reproduces (node visits / triangle tests match the
reference to the unit, which they cannot with a different tree), and -- where
/root/reference is present -- byte identity of the loader's arrays with the committed
fixture scenes/cornell_scene.npz.
"""
import hashlib
import os

import numpy as np
import pytest

from clrt import _native as N
from clrt import scene as S

REF = "/root/reference"
RT_FILE_NOT_FOUND = -1001  # rt_status.h


def _write(tmp_path, obj: str, mtl: str, name="m.obj"):
    p = tmp_path / name
    p.write_text(obj)
    (tmp_path / (name[:-4] + ".mtl")).write_text(mtl)
    return str(p)


MTL = """newmtl A
Kd 0.1 0.2 0.3
Ks 0.4 0.5 0.6
Ke 1 2 3
Ns 64
Ni 1.5
newmtl B
"""

VERTS = """v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
vt 0.25 0.5
vt 0.75 0.5
vt 0.75 1
vt 0.25 1
vn 0 0 1
vn 0 0 1
vn 0 0 1
vn 0 0 1
"""


def test_triangle_face_emits_two_triangles(tmp_path):
    """A 3-vertex face gives (1,2,3) from the fan loop plus the 'closing' (2,3,1)
    triangle (CLOBJloader.cpp:101-126): every triangle face is loaded twice."""
    p = _write(tmp_path, VERTS + "usemtl A\nf 1/1/1 2/2/2 3/3/3\n", MTL)
    s = S.load_obj(p, build=False)
    t = s.triangles
    assert t.shape[0] == 2
    pos = lambda i, v: tuple(t[i][v]["position"][:3])
    assert (pos(0, "v1"), pos(0, "v2"), pos(0, "v3")) == ((0, 0, 0), (1, 0, 0), (1, 1, 0))
    assert (pos(1, "v1"), pos(1, "v2"), pos(1, "v3")) == ((1, 0, 0), (1, 1, 0), (0, 0, 0))
    # uv = (vt.x, vt.y, 0) (CLshared_structs.hpp:32-35), normal from vn
    assert tuple(t[0]["v2"]["uv"][:3]) == (0.75, 0.5, 0.0)
    assert tuple(t[0]["v1"]["normal"][:3]) == (0.0, 0.0, 1.0)
    assert (t["mtlIndex"] == 0).all()


def test_quad_face_fan_plus_closing_triangle(tmp_path):
    p = _write(tmp_path, VERTS + "usemtl B\nf 1/1/1 2/2/2 3/3/3 4/4/4\n", MTL)
    t = S.load_obj(p, build=False).triangles
    assert t.shape[0] == 3  # (1,2,3), (2,3,4), closing (3,4,1)
    firsts = [tuple(t[i]["v1"]["position"][:3]) for i in range(3)]
    assert firsts == [(0, 0, 0), (1, 0, 0), (1, 1, 0)]
    assert tuple(t[2]["v3"]["position"][:3]) == (0, 0, 0)
    assert (t["mtlIndex"] == 1).all()


def test_material_fields_and_defaults(tmp_path):
    """Kd/Ks/Ke -> diffuse/specular/emission, Ns -> roughness, Ni -> ior; a material with
    no fields keeps CLMaterial()'s defaults (CLshared_structs.hpp:16)."""
    p = _write(tmp_path, VERTS + "usemtl A\nf 1/1/1 2/2/2 3/3/3\n", MTL)
    m = S.load_obj(p, build=False).materials
    assert m.shape[0] == 2
    np.testing.assert_array_equal(m[0]["diffuse"][:3], np.float32([0.1, 0.2, 0.3]))
    np.testing.assert_array_equal(m[0]["specular"][:3], np.float32([0.4, 0.5, 0.6]))
    np.testing.assert_array_equal(m[0]["emission"][:3], np.float32([1, 2, 3]))
    assert m[0]["roughness"] == np.float32(64) and m[0]["ior"] == np.float32(1.5)
    np.testing.assert_array_equal(m[1]["diffuse"][:3], np.float32([0.2] * 3))
    np.testing.assert_array_equal(m[1]["specular"][:3], np.float32([1] * 3))
    assert m[1]["roughness"] == np.float32(9999) and m[1]["ior"] == 0


def test_unknown_material_keeps_previous_index(tmp_path):
    """usemtl with an unknown name leaves materialIndex unchanged (CLOBJloader.cpp:65-75):
    before any match it is (unsigned)-1, which the launch then rejects."""
    p = _write(tmp_path, VERTS + "usemtl nope\nf 1/1/1 2/2/2 3/3/3\nusemtl B\nusemtl nope\n"
               "f 1/1/1 3/3/3 4/4/4\n", MTL)
    t = S.load_obj(p, build=False).triangles
    assert list(t["mtlIndex"]) == [0xFFFFFFFF, 0xFFFFFFFF, 1, 1]


def test_missing_files_and_bad_faces(tmp_path):
    with pytest.raises(N.RTError) as e:
        S.load_obj(str(tmp_path / "absent.obj"))
    assert e.value.code == RT_FILE_NOT_FOUND
    (tmp_path / "nomtl.obj").write_text(VERTS + "f 1/1/1 2/2/2 3/3/3\n")
    with pytest.raises(N.RTError) as e:
        S.load_obj(str(tmp_path / "nomtl.obj"))
    assert e.value.code == RT_FILE_NOT_FOUND  # the reference throws on a missing .mtl too
    p = _write(tmp_path, VERTS + "usemtl A\nf 1/1/1 9/9/9 3/3/3\n", MTL, name="bad.obj")
    with pytest.raises(N.RTError):
        S.load_obj(p)


def _check_bvh(sc):
    nodes, tris = sc.nodes, sc.triangles
    n = nodes.shape[0]
    covered = np.zeros(tris.shape[0], np.int32)
    p = np.stack([tris["v1"]["position"][:, :3], tris["v2"]["position"][:, :3],
                  tris["v3"]["position"][:, :3]], 1)
    seen = np.zeros(n, bool)
    stack = [0]
    while stack:
        i = stack.pop()
        seen[i] = True
        x = nodes[i]
        lo, hi = x["bmin"][:3], x["bmax"][:3]
        if x["nPrimitives"] > 0:
            a, b = int(x["offset"]), int(x["offset"]) + int(x["nPrimitives"])
            covered[a:b] += 1
            assert (p[a:b].reshape(-1, 3) >= lo).all() and (p[a:b].reshape(-1, 3) <= hi).all()
        else:
            c1, c2 = i + 1, int(x["offset"])  # DFS preorder: first child follows its parent
            assert i < c1 < c2 < n and x["axis"] <= 2
            for c in (c1, c2):
                assert (nodes[c]["bmin"][:3] >= lo).all() and (nodes[c]["bmax"][:3] <= hi).all()
            stack += [c2, c1]
    assert seen.all(), "unreachable nodes"
    assert (covered == 1).all(), "leaves must partition the triangle array"


def test_cornell_tree_matches_reference_probe(cornell):
    """72 triangles, 6 materials, 39 nodes, 20 leaves, <= 4 per leaf,
    depth 7 counted in levels (tree_stats counts edges from the root: 6)."""
    assert cornell.triangles.shape[0] == 72 and cornell.materials.shape[0] == 6
    assert cornell.nodes.shape[0] == 39
    st = cornell.tree_stats()
    assert st == {"max_depth": 6, "leaves": 20, "max_leaf_prims": 4}
    _check_bvh(cornell)


@pytest.mark.parametrize("max_prims", [1, 2, 4, 8, 255])
def test_bvh_invariants_any_leaf_size(cornell, max_prims):
    sc = S.build_bvh(cornell.triangles, cornell.materials, max_prims)
    _check_bvh(sc)
    # a leaf may hold more than max_prims: primitives with one shared centroid (every face
    # is loaded twice) cannot be split, and the SAH may prefer a leaf
    assert sc.tree_stats()["leaves"] >= 1


def test_build_is_a_permutation_of_the_input(cornell):
    z = np.load(S.CORNELL_NPZ, allow_pickle=False)
    src = z["triangles"].view(N.TRIANGLE_DTYPE)
    key = lambda a: sorted(bytes(r) for r in a.view(np.uint8).reshape(a.shape[0], -1))
    assert key(src) == key(cornell.triangles)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference scene files not present")
def test_loader_reproduces_committed_fixture():
    """Parsing the reference's own cornell.obj/.mtl gives the fixture's bytes (and hashes)."""
    z = np.load(S.CORNELL_NPZ, allow_pickle=False)
    s = S.load_obj(os.path.join(REF, "cornell.obj"), build=False)
    assert s.triangles.view(np.uint8).tobytes() == z["triangles"].tobytes()
    assert s.materials.view(np.uint8).tobytes() == z["materials"].tobytes()
    for key, fn in (("obj_sha256", "cornell.obj"), ("mtl_sha256", "cornell.mtl")):
        if key in z.files:
            h = hashlib.sha256(open(os.path.join(REF, fn), "rb").read()).digest()
            assert z[key].tobytes() == h


def test_binary_scene_cache_roundtrip(tmp_path, cornell):
    """rtsSaveScene / rtsLoadScene: byte-identical arrays back; corruption and
    truncation are RT_PARSE_ERROR, a missing file RT_FILE_NOT_FOUND."""
    p = str(tmp_path / "c.rtscene")
    S.save_scene(cornell, p)
    back = S.load_scene(p)
    for a, b in ((cornell.triangles, back.triangles), (cornell.nodes, back.nodes),
                 (cornell.materials, back.materials)):
        assert a.tobytes() == b.tobytes()
    raw = bytearray(open(p, "rb").read())
    raw[200] ^= 1
    bad = tmp_path / "bad.rtscene"
    bad.write_bytes(bytes(raw))
    with pytest.raises(N.RTError) as e:
        S.load_scene(str(bad))
    assert e.value.code == -1002
    (tmp_path / "short.rtscene").write_bytes(bytes(raw[:-9]))
    with pytest.raises(N.RTError) as e:
        S.load_scene(str(tmp_path / "short.rtscene"))
    assert e.value.code == -1002
    with pytest.raises(N.RTError) as e:
        S.load_scene(str(tmp_path / "none.rtscene"))
    assert e.value.code == RT_FILE_NOT_FOUND


def test_from_arrays_rejects_broken_trees(cornell):
    nodes = cornell.nodes.copy()
    nodes[0]["offset"] = 0  # second child before the first
    with pytest.raises(N.RTError):
        S.save_scene(S.Scene(cornell.triangles, nodes, cornell.materials), "/tmp/never_written.rtscene")
