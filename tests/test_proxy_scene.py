"""The bunny-class proxy (config 5): deterministic generation, loader/BVH structure, and
parity on the GPU through the global-memory scene path (3.3 MB of triangles, no LDS)."""
import hashlib
import os

import numpy as np
import pytest

from clrt import _native as N

PROXY_SHA256 = "c7455609c2012d07"  # prefix of the generated OBJ text (math-module trig, %.6f)


@pytest.fixture(scope="module")
def proxy():
    import clrt.proxy as P
    return P.bunny_proxy()


def test_proxy_is_deterministic_and_bunny_class(proxy):
    import clrt.proxy as P
    path = os.path.join(P.GEN_DIR, "bunny_proxy.obj")
    assert hashlib.sha256(open(path, "rb").read()).hexdigest().startswith(PROXY_SHA256)
    assert 65000 <= proxy.n_triangles <= 75000          # ~35k faces, doubled by the loader
    st = proxy.tree_stats()
    assert 40000 <= len(proxy.nodes) <= 60000 and st["max_depth"] >= 16
    assert st["max_leaf_prims"] <= 4
    # every triangle appears in exactly one leaf
    cover = np.zeros(proxy.n_triangles, np.int32)
    for n in proxy.nodes[proxy.nodes["nPrimitives"] > 0]:
        cover[n["offset"]:n["offset"] + n["nPrimitives"]] += 1
    assert (cover == 1).all()


def test_proxy_fills_default_camera(proxy, oracle_mod):
    _, ids, _, c = oracle_mod.render(proxy, 320, 180, light_bounces=1, want_hits=True)
    assert (ids >= 0).mean() > 0.8
    assert c["node_visits"] / c["rays"] > 20   # deep, divergent traversal


@pytest.mark.gpu
def test_proxy_pinned_bit_exact_vs_oracle(proxy, oracle_mod):
    from hip_helpers import HipRenderer, rgb
    W, H = 640, 360
    r = HipRenderer(proxy, W, H, math=N.MATH_PINNED, hits=True, stats=True)
    for f in (1, 2):
        r.frame(f, light_bounces=9)
    got = r.result()
    ids, _ = r.hits()
    st = r.k.stats()
    in_lds = r.k.scene_in_lds()
    r.close()
    assert not in_lds
    want = np.zeros((W * H, 4), np.float32)
    rays = visits = 0
    for f in (1, 2):
        want, wids, _, c = oracle_mod.render(proxy, W, H, frame_count=f, light_bounces=9, result=want,
                                             want_hits=True, threads=16)
        rays += c["rays"]
        visits += c["node_visits"]
    assert np.array_equal(ids, wids)  # primary hits of the last frame
    assert rgb(got).tobytes() == rgb(want).tobytes()
    assert st["rays"] == rays and st["node_visits"] == visits


@pytest.mark.gpu
@pytest.mark.parametrize("variant,math", [("strict", N.MATH_DEVICELIB), ("shipped", N.MATH_SHIPPED)])
def test_proxy_equals_live_reference(proxy, variant, math):
    """devicelib vs the strict reference build, shipped vs the default build: bit-exact on
    the global-memory scene path (70k triangles)."""
    import clref
    ok, why = clref.available()
    if not ok:
        pytest.skip(why)
    try:
        ref = clref.ReferenceKernel(variant)
    except RuntimeError as e:
        pytest.skip(str(e))
    from hip_helpers import HipRenderer, rgb
    W, H = 640, 360
    want = ref.render(proxy, W, H, frames=(1, 2), light_bounces=9)[:, :3]
    ids_r, t_r = ref.primary_hits(proxy, W, H)
    ref.close()
    r = HipRenderer(proxy, W, H, math=math)
    for f in (1, 2):
        r.frame(f, light_bounces=9)
    got = rgb(r.result())
    r.close()
    h = HipRenderer(proxy, W, H, math=math, hits=True)
    h.frame(1, light_bounces=1)
    ids, t = h.hits()
    h.close()
    assert np.array_equal(ids, ids_r)
    assert t.tobytes() == t_r.tobytes()
    assert got.tobytes() == want.tobytes()
