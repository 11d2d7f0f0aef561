"""Deterministic "bunny-class" proxy mesh (BASELINE.json config 5).

No Stanford bunny exists in the image and there is no network, so config 5 uses a
generated stand-in with the properties that matter for the hot path: ~35k triangle faces
(-> ~70k triangles after the reference loader doubles every face, CLOBJloader.cpp:101-126),
an irregular closed surface (a sphere displaced by a fixed sum of sinusoids, so the SAH
BVH is deep and unbalanced: ~48k nodes, depth in the 20s), framed to fill the default
camera's view (CLcamera.h:8-10: eye (0,-25,8.5) looking +y), faces written as `v/vt/vn`
triplets (the loader requires them, CLOBJloader.cpp:96) with outward counter-clockwise
winding (the kernel culls back faces, kernel_bvh.cl:116).

The OBJ is generated on demand into scenes/generated/ (git-ignored) and read back with the
product loader, so loading, BVH build and traversal are all exercised on it.
"""
from __future__ import annotations

import math
import os

import numpy as np

from .scene import Scene, load_obj, load_scene, save_scene

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GEN_DIR = os.path.join(_REPO, "scenes", "generated")


def _surface(theta: float, phi: float) -> float:
    """Radius of the displaced sphere at polar angle theta, azimuth phi (math-module trig,
    so the OBJ text is identical on every machine with the same libm)."""
    r = 7.0
    r += 0.9 * math.sin(3.0 * theta) * math.cos(2.0 * phi)
    r += 0.6 * math.sin(5.0 * theta + 1.3) * math.sin(3.0 * phi + 0.4)
    r += 0.35 * math.cos(9.0 * theta) * math.sin(7.0 * phi + 2.1)
    r += 0.2 * math.sin(17.0 * theta + 0.7) * math.cos(13.0 * phi)
    return r


def _point(theta: float, phi: float):
    r = _surface(theta, phi)
    return (r * math.sin(theta) * math.cos(phi) * 1.4, r * math.sin(theta) * math.sin(phi) * 0.8,
            r * math.cos(theta) * 1.1)


def write_bunny_proxy(obj_path: str, n_theta: int = 133, n_phi: int = 133) -> int:
    """Write the proxy OBJ + MTL; returns the number of triangle faces written."""
    center = np.array([0.0, -10.0, 8.5])
    th = [math.pi * i / (n_theta - 1) for i in range(n_theta)]
    ph = [2.0 * math.pi * j / n_phi for j in range(n_phi)]
    pos = np.array([[_point(t, f) for f in ph] for t in th]) + center
    # normals: central differences of the parametrisation
    e = 1e-4
    nrm = np.zeros_like(pos)
    for i, t in enumerate(th):
        for j, f in enumerate(ph):
            dt = np.subtract(_point(t + e, f), _point(t - e, f))
            dp = np.subtract(_point(t, f + e), _point(t, f - e))
            nrm[i, j] = np.cross(dt, dp)
    radial = pos - center
    bad = np.linalg.norm(nrm, axis=-1) < 1e-12
    nrm[bad] = radial[bad]
    nrm /= np.linalg.norm(nrm, axis=-1, keepdims=True)
    flip = (nrm * radial).sum(-1) < 0  # outward
    nrm[flip] *= -1.0

    # vertex ids: interior rings share the seam; poles are single vertices
    vid = np.full((n_theta, n_phi), -1, np.int64)
    verts, norms, uvs = [], [], []
    for i in range(n_theta):
        for j in range(n_phi):
            if (i == 0 or i == n_theta - 1) and j > 0:
                vid[i, j] = vid[i, 0]
                continue
            vid[i, j] = len(verts)
            verts.append(pos[i, j])
            norms.append(nrm[i, j])
            uvs.append((j / n_phi, i / (n_theta - 1)))
    faces = []
    for i in range(n_theta - 1):
        for j in range(n_phi):
            j2 = (j + 1) % n_phi
            a, b, c, d = vid[i, j], vid[i + 1, j], vid[i + 1, j2], vid[i, j2]
            for tri in ((a, b, c), (a, c, d)):
                if len(set(tri)) < 3:
                    continue
                faces.append(tri)
    verts = np.array(verts)
    # orient every face counter-clockwise seen from outside
    out = []
    for (a, b, c) in faces:
        n = np.cross(verts[b] - verts[a], verts[c] - verts[a])
        centroid = (verts[a] + verts[b] + verts[c]) / 3.0
        out.append((a, b, c) if np.dot(n, centroid - center) > 0 else (a, c, b))

    os.makedirs(os.path.dirname(os.path.abspath(obj_path)), exist_ok=True)
    mtl_path = obj_path[:-4] + ".mtl"
    with open(mtl_path, "w") as f:
        f.write("newmtl Proxy\nNs 64.0\nKd 0.70 0.62 0.55\nKs 0.30 0.30 0.30\nKe 0.0 0.0 0.0\nNi 1.0\n")
    with open(obj_path, "w") as f:
        f.write(f"mtllib {os.path.basename(mtl_path)}\no BunnyProxy\n")
        for v in verts:
            f.write(f"v {v[0]:.6f} {v[1]:.6f} {v[2]:.6f}\n")
        for (u, v) in uvs:
            f.write(f"vt {u:.6f} {v:.6f}\n")
        for nn in norms:
            f.write(f"vn {nn[0]:.6f} {nn[1]:.6f} {nn[2]:.6f}\n")
        f.write("usemtl Proxy\ns off\n")
        for (a, b, c) in out:
            f.write(f"f {a + 1}/{a + 1}/{a + 1} {b + 1}/{b + 1}/{b + 1} {c + 1}/{c + 1}/{c + 1}\n")
    return len(out)


def bunny_proxy(max_prims_in_node: int = 4, path: str | None = None, cache: bool = True) -> Scene:
    """Generate (if needed) and load the proxy through the product OBJ loader + SAH builder;
    the built arrays are kept in a binary scene cache next to the OBJ (rtsSaveScene)."""
    path = path or os.path.join(GEN_DIR, "bunny_proxy.obj")
    # several ranks (bench.py --gpus N) may generate at once: write to a private temporary
    # file and rename it into place, so a reader sees no file or a complete one
    tag = f".{os.getpid()}.tmp"
    if not os.path.exists(path):
        tmp_dir = os.path.join(os.path.dirname(os.path.abspath(path)), "tmp" + tag)
        tmp_obj = os.path.join(tmp_dir, os.path.basename(path))
        write_bunny_proxy(tmp_obj)  # OBJ + MTL with their final names, in a private directory
        os.replace(tmp_obj[:-4] + ".mtl", path[:-4] + ".mtl")
        os.replace(tmp_obj, path)
        os.rmdir(tmp_dir)
    cpath = f"{path[:-4]}.mp{max_prims_in_node}.rtscene"
    if cache and os.path.exists(cpath) and os.path.getmtime(cpath) >= os.path.getmtime(path):
        return load_scene(cpath, max_prims_in_node)
    sc = load_obj(path, max_prims_in_node)
    if cache:
        save_scene(sc, cpath + tag)
        os.replace(cpath + tag, cpath)
    return sc
