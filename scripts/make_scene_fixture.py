"""Generate scenes/cornell_scene.npz from the reference's own scene data files.

Runs HERE (where /root/reference exists): parses /root/reference/cornell.obj/.mtl with
the product loader (clrt.load_obj, a restatement of CLOBJloader.cpp:10-176) and stores
the parsed arrays (file order, before the BVH build) plus the SHA-256 of the two input
files.  GPU-box code loads this fixture instead of the reference files and builds the
BVH with the product builder; tests/test_scene.py checks, where the reference is
present, that loading the OBJ directly gives byte-identical arrays.
"""
import hashlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
import clrt  # noqa: E402

REF = "/root/reference"


def main():
    obj, mtl = os.path.join(REF, "cornell.obj"), os.path.join(REF, "cornell.mtl")
    s = clrt.load_obj(obj, build=False)
    out = os.path.join(REPO, "scenes", "cornell_scene.npz")
    np.savez_compressed(
        out,
        triangles=s.triangles.view(np.uint8),
        materials=s.materials.view(np.uint8),
        obj_sha256=np.frombuffer(hashlib.sha256(open(obj, "rb").read()).digest(), np.uint8),
        mtl_sha256=np.frombuffer(hashlib.sha256(open(mtl, "rb").read()).digest(), np.uint8),
    )
    print("wrote", out, s.triangles.shape, s.materials.shape)


if __name__ == "__main__":
    main()
