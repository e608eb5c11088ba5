"""The densify CLI's image ingest on the CPU: its JPEG decoder
(programs/densify/jpeg.cpp) against libjpeg-turbo's own decode of the same
files (tests/golden/jpeg_ingest.npz, made by tests/golden/make_golden_jpeg.py),
byte for byte -- the decode cv::imread performs for the reference
(modules/core/types.cpp:7-11)."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DENSIFY_DIR = os.path.join(ROOT, "programs", "densify")
TOOL = os.path.join(DENSIFY_DIR, "imgdecode")
GOLDEN = os.path.join(ROOT, "tests", "golden", "jpeg_ingest.npz")


@pytest.fixture(scope="module")
def tool():
    subprocess.run(["make", "-s", "-C", DENSIFY_DIR, "imgdecode"], check=True)
    return TOOL


def read_ppm(path: str) -> np.ndarray:
    data = open(path, "rb").read()
    parts = data.split(b"\n", 3)
    assert parts[0] == b"P6" and parts[2] == b"255"
    w, h = map(int, parts[1].split())
    return np.frombuffer(parts[3], dtype=np.uint8).reshape(h, w, 3)


def decode(tool, path, tmp_path):
    out = str(tmp_path / "out.ppm")
    r = subprocess.run([tool, str(path), out], capture_output=True, text=True)
    return r, (read_ppm(out)[:, :, ::-1] if r.returncode == 0 else None)


GOLD = np.load(GOLDEN)
CASES = sorted(k[: -len("__jpg")] for k in GOLD.files if k.endswith("__jpg"))


@pytest.mark.parametrize("name", CASES)
def test_jpeg_decode_equals_libjpeg_turbo(tool, tmp_path, name):
    src = tmp_path / (name + ".jpg")
    src.write_bytes(GOLD[name + "__jpg"].tobytes())
    r, bgr = decode(tool, src, tmp_path)
    assert r.returncode == 0, r.stderr
    want = GOLD[name + "__bgr"]
    assert bgr.shape == want.shape
    diff = np.abs(bgr.astype(int) - want.astype(int))
    assert diff.max() == 0, f"{name}: {int((diff > 0).sum())} bytes differ, max {int(diff.max())}"


def test_jpeg_fixture_covers_the_layouts():
    """the fixture holds every layout the decoder claims: 4:4:4 / 4:2:2 / 4:2:0,
    gray, restart markers, progressive, EXIF orientation, odd and tiny sizes"""
    for key in ("444", "422", "420", "gray", "restart", "progressive", "exif", "tiny", "one_1x1"):
        assert any(key in c for c in CASES), key


def test_png_and_jpeg_of_same_pixels_decode_equal(tool, tmp_path):
    """a PNG holding the JPEG's decoded pixels loads to the same BGR8 image"""
    zlib = pytest.importorskip("zlib")
    name = "q75_420"
    want = GOLD[name + "__bgr"]
    h, w, _ = want.shape
    rgb = want[:, :, ::-1]
    raw = b"".join(b"\x00" + rgb[y].tobytes() for y in range(h))

    def chunk(t, d):
        import struct
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    import struct
    png = (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) +
           chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b""))
    (tmp_path / "a.png").write_bytes(png)
    r, got = decode(tool, tmp_path / "a.png", tmp_path)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(got, want)


def test_unsupported_and_corrupt_jpegs_fail_loudly(tool, tmp_path):
    data = bytearray(GOLD["q90_444__jpg"].tobytes())
    bad = tmp_path / "trunc.jpg"
    bad.write_bytes(bytes(data[: len(data) // 3]))
    r, _ = decode(tool, bad, tmp_path)
    assert r.returncode != 0 and "trunc.jpg" in r.stderr
    # a 12-bit frame header (SOF1 with P = 12) is refused with a message
    i = data.index(b"\xff\xc0")
    data[i + 4] = 12
    tw = tmp_path / "twelve.jpg"
    tw.write_bytes(bytes(data))
    r, _ = decode(tool, tw, tmp_path)
    assert r.returncode != 0 and "8-bit" in r.stderr
    # a DC Huffman table with a magnitude category above 15 (libjpeg
    # rejects it when it builds the table): the first DHT of class 0 gets
    # symbol 200 in place of its last symbol
    data = bytearray(GOLD["q90_444__jpg"].tobytes())
    i = data.index(b"\xff\xc4")
    assert data[i + 4] >> 4 == 0  # class 0 (DC)
    nv = sum(data[i + 5:i + 21])
    data[i + 21 + nv - 1] = 200
    bd = tmp_path / "baddc.jpg"
    bd.write_bytes(bytes(data))
    r, _ = decode(tool, bd, tmp_path)
    assert r.returncode != 0 and "DC symbol" in r.stderr, r.stderr
