"""The `shipped` math mode pinned to the reference kernel as the OpenCL RUNTIME builds it.

The reference host JIT-compiles kernel_bvh.cl with program.build(" -I . ")
(/root/reference/CLutils.cpp:52-66).  oracle/_ref/kernel_bvh_shipped.co -- from which the shipped
policy (csrc/rt_math.hpp: contraction sites, 2.5-ulp division, 3-ulp sqrt) was read -- is a clang
`-x cl -O3` build with the compiler's defaults.  This file closes the gap between the two: the
image's own OpenCL runtime builds the unmodified source for an offline gfx950 device
(oracle/offline_build.c, cl_amd_offline_devices: the same clCreateProgramWithSource +
clBuildProgram path as the reference, no GPU needed), and

  CPU: the runtime's KernelEntry is the same code whether it builds kernel_bvh.cl alone (the
       reference's program) or the ref_entry.cl harness around it; it uses exactly the
       floating-point operation kinds of the clang build (fused multiply-adds where the source
       contracts, the rcp/frexp/ldexp division and the scaled v_sqrt -- no IEEE div_scale/fixup
       expansion of `/` beyond the clang build's own).  The instruction texts differ: the runtime
       links with -amdgpu-prelink/internalize and preloads kernel arguments, so registers and
       schedule differ and a few blocks are duplicated differently (recorded below);
  GPU: the runtime-built kernel, run through the system OpenCL runtime, produces the same bits as
       the clang build and as the HIP shipped mode -- primary hit IDs and t, and radiance over
       many bounces and frames (every transcendental and division site exercised).
"""
import os
import re
import subprocess

import numpy as np
import pytest

from clrt import _native as N
from hip_helpers import HipRenderer, rgb
from ref_compare import bits_differ, rel_err

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = os.path.join(REPO, "oracle", "_ref")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def _co(name):
    p = os.path.join(REF_DIR, name)
    if not os.path.exists(p):
        pytest.skip(f"{p} not built (make -C oracle ref: needs /root/reference and the OpenCL runtime)")
    return p


def _kernel_entry_insts(path):
    """KernelEntry's instructions (mnemonic + operands), trailing s_nop padding dropped."""
    out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", path], capture_output=True, text=True,
                         check=True).stdout
    lines, on = [], False
    for ln in out.splitlines():
        if re.match(r"^[0-9a-f]+ <KernelEntry>:", ln):
            on = True
            continue
        if on and re.match(r"^[0-9a-f]+ <", ln):
            break
        if on:
            ln = re.sub(r"//.*", "", ln).strip()
            if ln:
                lines.append(ln)
    while lines and lines[-1].startswith("s_nop"):
        lines.pop()
    assert lines, f"no KernelEntry in {path}"
    return lines


def _fp_kinds(insts):
    """floating-point operation kinds (encoding suffix dropped) -> count"""
    kinds = {}
    for i in insts:
        op = re.sub(r"_e(32|64)$", "", i.split()[0])
        if op.startswith("v_") and re.search(r"f(16|32|64)", op):
            kinds[op] = kinds.get(op, 0) + 1
    return kinds


def test_runtime_kernel_is_the_reference_program():
    """The harness (ref_entry.cl, + PrimaryHitEntry) leaves the runtime's KernelEntry as it
    builds it for the reference's own program."""
    a = _kernel_entry_insts(_co("kernel_bvh_runtime_ref.co"))
    b = _kernel_entry_insts(_co("kernel_bvh_runtime.co"))
    assert a == b


def test_runtime_build_uses_the_shipped_operation_kinds():
    rt = _fp_kinds(_kernel_entry_insts(_co("kernel_bvh_runtime_ref.co")))
    cl = _fp_kinds(_kernel_entry_insts(_co("kernel_bvh_shipped.co")))
    assert set(rt) == set(cl), (sorted(set(rt) ^ set(cl)))
    # contraction (fp-contract=on) and the OpenCL-accuracy division / sqrt in both builds; the
    # correctly rounded forms' div_scale/div_fmas/div_fixup appear once in both (a double
    # division the clang build keeps too)
    for k in ("v_fma_f32", "v_fmac_f32", "v_rcp_f32", "v_frexp_mant_f32", "v_ldexp_f32", "v_sqrt_f32"):
        assert rt.get(k, 0) > 0 and cl.get(k, 0) > 0, k
    assert rt.get("v_div_scale_f32", 0) == cl.get("v_div_scale_f32", 0)
    # the recorded count differences are duplicated blocks, not different arithmetic (the GPU
    # tests below compare the bits)
    diff = {k: cl[k] - rt[k] for k in cl if cl[k] != rt[k]}
    assert sum(abs(v) for v in diff.values()) < 0.05 * sum(cl.values()), diff


# ---- GPU: the runtime-built reference, live -------------------------------------------------
def _open(variant):
    import clref
    ok, why = clref.available()
    if not ok:
        pytest.skip(why)
    if not os.path.exists(clref.VARIANTS[variant]):
        pytest.skip(f"{clref.VARIANTS[variant]} not built")
    try:
        return clref.ReferenceKernel(variant)
    except RuntimeError as e:
        pytest.skip(f"no OpenCL GPU device for the reference: {e}")


@pytest.fixture(scope="module")
def live_runtime():
    r = _open("runtime")
    yield r
    r.close()


@pytest.fixture(scope="module")
def live_shipped_co():
    r = _open("shipped")
    yield r
    r.close()


def _hip(scene, W, H, frames, bounces, hits=False):
    r = HipRenderer(scene, W, H, math=N.MATH_SHIPPED, hits=hits)
    for f in frames:
        r.frame(f, light_bounces=bounces)
    out = rgb(r.result())
    h = r.hits() if hits else None
    r.close()
    return out, h


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(512, 512), (1920, 1080)])
def test_shipped_primary_hits_equal_runtime_built_reference(cornell, live_runtime, W, H):
    ids_r, t_r = live_runtime.primary_hits(cornell, W, H)
    _, (ids, t) = _hip(cornell, W, H, [1], 1, hits=True)
    assert np.array_equal(ids, ids_r), f"{(ids != ids_r).sum()} ids differ"
    assert bits_differ(t, t_r) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,bounces,frames", [(1920, 1080, 2, 1), (512, 512, 9, 8), (3840, 2160, 9, 2)])
def test_shipped_equals_runtime_built_reference(cornell, live_runtime, W, H, bounces, frames):
    want = live_runtime.render(cornell, W, H, frames=range(1, frames + 1), light_bounces=bounces)[:, :3]
    got, _ = _hip(cornell, W, H, range(1, frames + 1), bounces)
    nd = bits_differ(got, want)
    assert nd == 0, f"{nd} words differ, max rel {rel_err(got, want).max():.3g}"


@pytest.mark.gpu
def test_runtime_build_equals_clang_build(cornell, live_runtime, live_shipped_co):
    """The clang build the shipped policy was read from and the runtime's own build: same bits,
    including light types 1 and 2 (the point light's double-precision attenuation)."""
    for lt in (0, 1, 2):
        a = live_runtime.render(cornell, 640, 360, frames=range(1, 5), light_bounces=9, light_type=lt)
        b = live_shipped_co.render(cornell, 640, 360, frames=range(1, 5), light_bounces=9, light_type=lt)
        assert bits_differ(a[:, :3], b[:, :3]) == 0, lt
