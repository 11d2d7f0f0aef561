"""CPU: the output/format step (include/rt_image.h) -- what the reference shows through its
GL_RGBA32F texture (CLRaytracer.cpp:25-26, :64-67), written to PPM / PNG instead."""
import struct
import zlib

import numpy as np
import pytest

from clrt import RTError
from clrt import image


def _buf(W, H, seed=3):
    rng = np.random.default_rng(seed)
    px = rng.uniform(-0.2, 1.2, size=(H * W, 4)).astype(np.float32)
    px[0, 0] = np.nan
    px[1, 1] = np.inf
    px[2, 2] = 0.5 / 255.0  # rounds up to 1
    return px


def _expected(px, W, H):
    v = px[:, :3].reshape(H, W, 3)[::-1]  # row 0 of the buffer is the bottom of the picture
    with np.errstate(invalid="ignore"):
        c = np.where(v > 0, np.minimum(v, 1.0), 0.0)
        out = np.floor(c.astype(np.float32) * np.float32(255.0) + np.float32(0.5))
    out = np.where(v >= 1.0, 255, out)
    return out.astype(np.uint8)


def test_to_rgb8_clamps_rounds_and_flips():
    W, H = 7, 5
    px = _buf(W, H)
    got = image.to_rgb8(px, W, H)
    assert got.shape == (H, W, 3)
    np.testing.assert_array_equal(got, _expected(px, W, H))
    assert got[H - 1, 0, 0] == 0          # NaN -> 0
    assert got[H - 1, 1, 1] == 255        # inf -> 255


def test_png_roundtrip(tmp_path):
    W, H = 300, 257  # > 65535 raw bytes: several stored deflate blocks
    px = _buf(W, H, seed=5)
    p = str(tmp_path / "a.png")
    image.write_png(p, px, W, H)
    b = open(p, "rb").read()
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, {}
    while pos < len(b):
        n, = struct.unpack(">I", b[pos:pos + 4])
        typ, data = b[pos + 4:pos + 8], b[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", b[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + data) & 0xffffffff
        chunks.setdefault(typ, b"")
        chunks[typ] += data
        pos += 12 + n
    w, h, depth, ctype, comp, filt, inter = struct.unpack(">IIBBBBB", chunks[b"IHDR"])
    assert (w, h, depth, ctype, comp, filt, inter) == (W, H, 8, 2, 0, 0, 0)
    raw = zlib.decompress(chunks[b"IDAT"])  # also checks the Adler-32
    rows = np.frombuffer(raw, np.uint8).reshape(H, 1 + 3 * W)
    assert (rows[:, 0] == 0).all()
    np.testing.assert_array_equal(rows[:, 1:].reshape(H, W, 3), _expected(px, W, H))
    assert b"IEND" in chunks


def test_ppm(tmp_path):
    W, H = 9, 4
    px = _buf(W, H, seed=9)
    p = str(tmp_path / "a.ppm")
    image.write_ppm(p, px, W, H)
    b = open(p, "rb").read()
    head = b"P6\n%d %d\n255\n" % (W, H)
    assert b.startswith(head)
    np.testing.assert_array_equal(np.frombuffer(b[len(head):], np.uint8).reshape(H, W, 3), _expected(px, W, H))


def test_errors(tmp_path):
    with pytest.raises(ValueError):
        image.write_png(str(tmp_path / "x.png"), np.zeros(5, np.float32), 2, 2)
    with pytest.raises(RTError):
        image.write_png(str(tmp_path / "no" / "dir.png"), np.zeros((4, 4), np.float32), 2, 2)


# ---- checkpoint / resume of the accumulation buffer (rtiSaveAccum / rtiLoadAccum) ----------------
def test_accum_checkpoint_round_trip(tmp_path):
    W, H = 13, 9
    px = _buf(W, H, seed=5)
    px[:, 3] = np.arange(W * H, dtype=np.float32)  # the 4th lane travels too (16-byte stride)
    p = str(tmp_path / "a.rtaccum")
    image.save_accum(p, px, W, H, 5)
    got, nf = image.load_accum(p)
    assert nf == 5
    assert got.tobytes() == px.tobytes()  # NaN / inf bits included


def test_accum_checkpoint_rejects_damage(tmp_path):
    W, H = 4, 3
    p = tmp_path / "a.rtaccum"
    image.save_accum(str(p), _buf(W, H), W, H, 2)
    raw = bytearray(p.read_bytes())
    raw[40] ^= 1  # a pixel bit
    bad = tmp_path / "bad.rtaccum"
    bad.write_bytes(bytes(raw))
    with pytest.raises(RTError):
        image.load_accum(str(bad))
    short = tmp_path / "short.rtaccum"
    short.write_bytes(p.read_bytes()[:-9])
    with pytest.raises(RTError):
        image.load_accum(str(short))
    with pytest.raises(RTError):
        image.load_accum(str(tmp_path / "missing.rtaccum"))
