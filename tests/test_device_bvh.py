"""GPU: device-side BVH build (rtBuildBVH).

The device builder writes the reference's node contract (CLBVHnode.cpp:161-183) but a
different tree than the host SAH build (host/scene.cpp, the reference's algorithm), so:
  * structure: depth-first layout, leaves partition the (permuted) triangle array, bounds
    contain their children and triangles, leaf sizes <= maxPrimitivesInNode;
  * parity is per geometry: rendering the device-built arrays is bit-exact with the CPU
    oracle rendering the same arrays (pinned math), and close to the SAH-built scene's image
    (the Cornell OBJ holds every face twice, so ties may pick the other copy).
"""
import time

import numpy as np
import pytest

from clrt import _native as N
from clrt import scene as S
from hip_helpers import HipRenderer, rgb
from ref_compare import rel_err
from test_scene import _check_bvh

pytestmark = pytest.mark.gpu


def _file_order_cornell():
    z = np.load(S.CORNELL_NPZ, allow_pickle=False)
    return z["triangles"].view(N.TRIANGLE_DTYPE), z["materials"].view(N.MATERIAL_DTYPE)


def _same_multiset(a, b):
    key = lambda x: sorted(bytes(r) for r in x.view(np.uint8).reshape(x.shape[0], -1))
    return key(a) == key(b)


METHODS = ["ploc", "lbvh"]


@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("max_prims", [1, 2, 4, 8])
def test_device_bvh_structure(max_prims, method):
    tris, mats = _file_order_cornell()
    sc = S.build_bvh_device(tris, mats, max_prims, method=method)
    _check_bvh(sc)
    leaf = sc.nodes["nPrimitives"]
    assert leaf.max() <= max_prims
    assert sc.nodes.shape[0] <= 2 * tris.shape[0] - 1
    assert _same_multiset(sc.triangles, tris)


@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("n", [1, 3])
def test_device_bvh_single_leaf(n, method):
    tris, mats = _file_order_cornell()
    sc = S.build_bvh_device(tris[:n], mats, 4, method=method)
    # n <= max_prims: one leaf, for both builders (PLOC collapses every subtree of <= max_prims
    # triangles; only an RT_PLOC_SAH_LEAVES build, off by default, lets the SAH keep it split)
    assert sc.nodes.shape[0] == 1 and sc.nodes[0]["nPrimitives"] == n
    assert sc.nodes["nPrimitives"].sum() == n
    _check_bvh(sc)


@pytest.mark.parametrize("method", METHODS)
def test_device_bvh_render_bit_exact_vs_oracle(oracle_mod, method):
    tris, mats = _file_order_cornell()
    sc = S.build_bvh_device(tris, mats, 4, method=method)
    W, H = 160, 90
    r = HipRenderer(sc, W, H, stats=True)
    for f in (1, 2):
        r.frame(f, light_bounces=9)
    got = r.result()
    st = r.k.stats()
    r.close()
    want = np.zeros((W * H, 4), np.float32)
    counts = {"node_visits": 0, "tri_tests": 0}
    for f in (1, 2):
        want, _, _, c = oracle_mod.render(sc, W, H, frame_count=f, light_bounces=9, result=want, threads=16)
        for k in counts:
            counts[k] += c[k]
    a, b = rgb(got), rgb(want)
    assert (a.view(np.uint32) == b.view(np.uint32)).all()
    assert (st["node_visits"], st["tri_tests"]) == (counts["node_visits"], counts["tri_tests"])


@pytest.mark.parametrize("method", METHODS)
def test_device_bvh_bunny_matches_sah_image(method):
    """70k-triangle proxy: the device tree renders the same geometry as the SAH tree."""
    from clrt import proxy
    host = proxy.bunny_proxy()
    raw = S.load_obj(proxy.os.path.join(proxy.GEN_DIR, "bunny_proxy.obj"), build=False)
    t0 = time.perf_counter()
    dev = S.build_bvh_device(raw.triangles, raw.materials, 4, method=method)
    build_s = time.perf_counter() - t0
    _check_bvh(dev)
    assert _same_multiset(dev.triangles, host.triangles)
    W, H = 256, 144
    imgs = []
    for sc in (host, dev):
        r = HipRenderer(sc, W, H, math=N.MATH_DEVICELIB, hits=True)
        r.frame(1, light_bounces=1)
        imgs.append((rgb(r.result()), r.hits()[0], None))
        r.close()
    (a, ida, _), (b, idb, _) = imgs

    def face_keys(sc):  # geometric identity of a triangle (the loader's two copies share it)
        pos = np.stack([sc.triangles[v]["position"][:, :3] for v in ("v1", "v2", "v3")], axis=1)
        return [tuple(sorted(map(tuple, q.tolist()))) for q in pos]

    kh, kd = face_keys(host), face_keys(dev)
    fa = [kh[i] if i >= 0 else None for i in ida.ravel()]
    fb = [kd[i] if i >= 0 else None for i in idb.ravel()]
    agree = np.mean([x == y for x, y in zip(fa, fb)])
    assert agree > 0.999, agree                      # the same face is hit
    rel = rel_err(a, b).max(axis=-1)
    assert (rel > 1e-4).mean() < 0.005               # radiance: last-bit differences from ties
    same = (a.view(np.uint32) == b.view(np.uint32)).all(axis=-1).mean()
    print(f"device {method} build of {raw.triangles.shape[0]} triangles: {build_s * 1e3:.1f} ms incl. transfers; "
          f"same face {agree:.5f}; {same:.4f} of pixels bit-identical to the SAH tree's image")


@pytest.mark.parametrize("method", [N.BVH_PLOC, N.BVH_LBVH])
@pytest.mark.parametrize("max_prims", [1, 4])
def test_device_bvh_buffers_bind_to_kernel_entry_as_they_are(oracle_mod, max_prims, method):
    """rt_hip.h's flow for rtBuildBVH: the triangle and node buffers it wrote are bound to
    KernelEntry directly -- the node buffer keeps its 2n-1 records (the tree is the first
    `count`, the rest unused) -- and the render equals the oracle's on the tree read back."""
    import clrt
    tris, mats = _file_order_cornell()
    n = tris.shape[0]
    W, H = 128, 96
    ctx = clrt.CLContext(0)
    tb = ctx.create_buffer(N.MEM_READ_WRITE | N.MEM_COPY_HOST_PTR, tris.nbytes, tris)
    nb = ctx.create_buffer(N.MEM_READ_WRITE, (2 * n - 1) * N.NODE_DTYPE.itemsize)
    mb = ctx.create_buffer(N.MEM_READ_ONLY | N.MEM_COPY_HOST_PTR, mats.nbytes, mats)
    count = ctx.BuildBVH(tb, n, max_prims, nb, method)
    assert (max_prims == 1) == (count == 2 * n - 1)
    out = ctx.create_buffer(N.MEM_WRITE_ONLY, W * H * 16)
    k = clrt.CLKernel(ctx)
    for slot, b in ((N.BUFFER_OUT, out), (N.BUFFER_SCENE, tb), (N.BUFFER_NODE, nb), (N.BUFFER_MATERIAL, mb)):
        k.set_buffer(slot, b)
    k.set_math_mode(N.MATH_PINNED)
    k.set_int(N.WIDTH, W)
    k.set_int(N.HEIGHT, H)
    k.set_int(N.LIGHT_BOUNCES, 4)
    k.set_int(N.LIGHT_TYPE, 0)
    k.set_float(N.SKYBOX_INTENSITY, 1.0)
    k.set_uint(N.FRAME_SEED, 0)
    for slot, v in zip((N.CAMERA_POS, N.CAMERA_FRONT, N.CAMERA_UP), ((0.0, -25.0, 8.5), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0))):
        k.set_float3(slot, v)
    k.set_uint(N.FRAME_COUNT, 1)
    ctx.ExecuteKernel(k, W * H)
    got = np.zeros((W * H, 4), np.float32)
    ctx.ReadBuffer(out, got, blocking=True)
    t_dev = np.empty_like(tris)
    n_dev = np.empty(count, N.NODE_DTYPE)
    ctx.ReadBuffer(tb, t_dev, blocking=True)
    ctx.ReadBuffer(nb, n_dev, n_dev.nbytes, blocking=True)
    for b in (tb, nb, mb, out):
        b.release()
    k.release()
    ctx.release()
    sc = S.Scene(t_dev, n_dev, mats, max_prims)
    want, _, _, _ = oracle_mod.render(sc, W, H, frame_count=1, light_bounces=4, threads=16)
    assert (rgb(got).view(np.uint32) == rgb(want).view(np.uint32)).all()


def _sah_cost(sc):
    """Surface-area-heuristic cost of a depth-first node array (interior 1, triangle test 1 per
    triangle), relative to the root box: the expected work of a random ray that hits the root."""
    lo, hi = sc.nodes["bmin"][:, :3].astype(np.float64), sc.nodes["bmax"][:, :3].astype(np.float64)
    d = np.maximum(hi - lo, 0.0)
    area = 2.0 * (d[:, 0] * d[:, 1] + d[:, 1] * d[:, 2] + d[:, 2] * d[:, 0])
    cnt = sc.nodes["nPrimitives"].astype(np.float64)
    return float(np.sum(area * np.where(cnt > 0, cnt, 1.0)) / area[0])


def test_device_bvh_ploc_tree_beats_lbvh():
    """PLOC clusters by surface area: on the 70k-triangle proxy its tree's SAH cost is well below
    the linear BVH's and within reach of the host SAH build (the reference's algorithm)."""
    from clrt import proxy
    host = proxy.bunny_proxy()
    raw = S.load_obj(proxy.os.path.join(proxy.GEN_DIR, "bunny_proxy.obj"), build=False)
    c = {m: _sah_cost(S.build_bvh_device(raw.triangles, raw.materials, 4, method=m)) for m in METHODS}
    c["host_sah"] = _sah_cost(host)
    print("SAH cost:", {k: round(v, 2) for k, v in c.items()})
    assert c["ploc"] < 0.9 * c["lbvh"], c
    assert c["ploc"] < 1.3 * c["host_sah"], c


@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("case", ["identical", "coplanar_grid", "random_soup"])
def test_device_bvh_degenerate_and_large_inputs(oracle_mod, method, case):
    """Inputs that stress the builders: 2,000 copies of one triangle (every Morton code and every
    PLOC cost ties: the pairing fallback), a flat grid of 20,000 triangles in one plane (zero-volume
    boxes), and a 150,000-triangle random soup.  The tree keeps the node contract and a render of it
    is bit-exact with the oracle rendering the same arrays."""
    tris, mats = _file_order_cornell()
    rng = np.random.default_rng(7)
    if case == "identical":
        out = np.repeat(tris[10:11], 2000)
    elif case == "coplanar_grid":
        g = 100
        xs, ys = np.meshgrid(np.linspace(-5, 5, g + 1)[:-1], np.linspace(-5, 5, g + 1)[:-1])
        out = np.repeat(tris[:1], 2 * g * g)
        d = 10.0 / g
        for k, (dx0, dy0, dx1, dy1, dx2, dy2) in enumerate(((0, 0, d, 0, 0, d), (d, 0, d, d, 0, d))):
            sl = out[k::2]
            sl["v1"]["position"][:, 0], sl["v1"]["position"][:, 1] = xs.ravel() + dx0, ys.ravel() + dy0
            sl["v2"]["position"][:, 0], sl["v2"]["position"][:, 1] = xs.ravel() + dx1, ys.ravel() + dy1
            sl["v3"]["position"][:, 0], sl["v3"]["position"][:, 1] = xs.ravel() + dx2, ys.ravel() + dy2
            for v in ("v1", "v2", "v3"):
                sl[v]["position"][:, 2] = 0.0
            out[k::2] = sl
    else:
        out = np.repeat(tris[:1], 150_000)
        c = rng.uniform(-6, 6, (out.shape[0], 3)).astype(np.float32) + np.float32([0, 0, 6])
        for v in ("v1", "v2", "v3"):
            out[v]["position"][:, :3] = c + rng.normal(0, 0.15, (out.shape[0], 3)).astype(np.float32)
    out["mtlIndex"] = 1
    sc = S.build_bvh_device(out, mats, 4, method=method)
    _check_bvh(sc)
    assert sc.nodes["nPrimitives"].max() <= 4
    assert _same_multiset(sc.triangles, out)
    W, H = 64, 48
    r = HipRenderer(sc, W, H)
    r.frame(1, light_bounces=3)
    got = r.result()
    r.close()
    want, _, _, _ = oracle_mod.render(sc, W, H, frame_count=1, light_bounces=3,
                                      result=np.zeros((W * H, 4), np.float32), threads=16)
    assert (rgb(got).view(np.uint32) == rgb(want).view(np.uint32)).all()
