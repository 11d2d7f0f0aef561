"""Comparison helpers between our outputs and the reference kernel's (fixtures or live)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def face_ids(scene):
    """Canonical face per triangle: the loader emits every OBJ triangle twice with rotated
    vertices (CLOBJloader.cpp:101-126); both copies map to one face id (the smallest
    triangle index with the same vertex-position set)."""
    pos = np.stack([scene.triangles[v]["position"][:, :3] for v in ("v1", "v2", "v3")], axis=1)
    keys = [tuple(sorted(map(tuple, p.tolist()))) for p in pos]
    first = {}
    out = np.empty(len(keys), np.int64)
    for i, k in enumerate(keys):
        out[i] = first.setdefault(k, i)
    return out


def map_faces(ids, faces):
    return np.where(ids >= 0, faces[np.maximum(ids, 0)], -1)


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    d = np.abs(a - b)
    m = np.maximum(np.abs(a), np.abs(b))
    with np.errstate(invalid="ignore", divide="ignore"):
        r = np.where(m > 0, d / m, 0.0)
    return r


def bits_differ(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.uint32).ravel()
    b = np.ascontiguousarray(b, np.float32).view(np.uint32).ravel()
    return int((a != b).sum())
