"""Frame output: rtow_write_bmp against BMP files the reference's own writer
(winDIBbitmap.cpp:20-168) produced (tests/golden/make_bmp_golden.py), and
the PPM writer's layout."""
import json
import os

import numpy as np
import pytest

import rtow

BMP = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bmp")
CASES = json.load(open(os.path.join(BMP, "manifest.json")))


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_bmp_matches_reference_writer(case, tmp_path):
    raw = np.fromfile(os.path.join(BMP, case["name"] + ".raw"), dtype=np.uint8)
    out = str(tmp_path / "out.bmp")
    rtow.write_bmp(out, raw, case["width"], case["height"], case["bpp"])
    with open(out, "rb") as f, open(os.path.join(BMP, case["name"] + ".bmp"), "rb") as g:
        assert f.read() == g.read()


def test_bmp_rejects_inconsistent_sizes(tmp_path):
    with pytest.raises(rtow.RtowError):
        rtow.write_bmp(str(tmp_path / "x.bmp"), np.zeros(10, np.uint8), 4, 4, 32)
    with pytest.raises(rtow.RtowError):
        rtow.write_bmp(str(tmp_path / "x.bmp"), np.zeros(48, np.uint8), 4, 4, 12)
    with pytest.raises(rtow.RtowError):
        rtow.write_bmp(str(tmp_path / "nodir" / "x.bmp"), np.zeros(64, np.uint8), 4, 4, 32)


def test_ppm_is_rgb_top_down(tmp_path):
    bgra = np.zeros((2, 3, 4), np.uint8)
    bgra[0, 0] = (1, 2, 3, 0)   # top-left: B G R A
    bgra[1, 2] = (10, 20, 30, 0)
    out = str(tmp_path / "x.ppm")
    rtow.write_ppm(out, bgra)
    data = open(out, "rb").read()
    hdr = b"P6\n3 2\n255\n"
    assert data.startswith(hdr)
    px = np.frombuffer(data[len(hdr):], np.uint8).reshape(2, 3, 3)
    assert tuple(px[0, 0]) == (3, 2, 1) and tuple(px[1, 2]) == (30, 20, 10)
