"""The host layout builder (csrc/rtow_layout.cpp, buildLayout) on the CPU.

rtow_scene_check with RTOW_LAYOUT_DUMP writes every array rtow_scene_upload
would copy to the device, so these tests see exactly what the kernels would
read, without a GPU.
"""
import os

import numpy as np

import rtow
import scene_io as sio

TEX_CONSTANT, TEX_CHECKER, TEX_NOISE = 1, 2, 3


def _dump(scene, tmp_path, tree="sah"):
    path = str(tmp_path / "layout.bin")
    old = {k: os.environ.get(k) for k in ("RTOW_LAYOUT_DUMP", "RTOW_BVH")}
    os.environ["RTOW_LAYOUT_DUMP"] = path
    if tree == "ref":
        os.environ["RTOW_BVH"] = "ref"
    else:
        os.environ.pop("RTOW_BVH", None)
    try:
        sio.scene_check(scene)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return open(path, "rb").read()


def test_checker_reserved_field_never_reaches_the_device(tmp_path):
    """DTex::c is the device's TEX_FLAT flag, rtow_texture::c is
    unused for a CheckerTexture (include/rtow.h).  A caller's nonzero c on a
    checker -- one of two constants (flattened anyway) and one whose child is
    a noise texture (never flattened) -- must give the layout of c = 0."""
    d = sio.scene_dict(rtow.Scene.build("random_ned", n=100, image="synthetic"))
    tex = d["textures"]
    checkers = np.flatnonzero(tex["kind"] == TEX_CHECKER)
    assert checkers.size >= 1
    noise = np.flatnonzero(tex["kind"] == TEX_NOISE)
    assert noise.size >= 1
    # a second checker: odd squares noise, even squares the first checker's odd colour
    extra = np.zeros(1, tex.dtype)
    extra[0]["kind"], extra[0]["a"], extra[0]["b"] = TEX_CHECKER, noise[0], tex[checkers[0]]["a"]
    d["textures"] = np.concatenate([tex, extra])
    mats = d["materials"].copy()
    uses = np.flatnonzero(mats["texture"] == checkers[0])
    assert uses.size >= 1
    mats[uses[0]]["texture"] = len(tex)  # one material renders through the new checker
    d["materials"] = mats
    clean = _dump(sio.ArrayScene(d), tmp_path)
    dirty = dict(d)
    dirty["textures"] = d["textures"].copy()
    dirty["textures"]["c"][dirty["textures"]["kind"] == TEX_CHECKER] = 0xdeadbeef
    assert _dump(sio.ArrayScene(dirty), tmp_path) == clean


def test_large_grid_is_still_a_grid(capfd):
    """a grid table larger than the MODE 8 kernel's LDS staging
    (GRID_LDS_WORDS = 512 packed words) was dropped back to tree traversal.
    final_ned with a 32 x 32 ground (1024 cells + 32 rows) keeps its grid
    (walked from global memory by the STACK 20 kernel, tests/test_grid.py),
    and so does the book's 20 x 20 (420 words, staged in LDS)."""
    old = os.environ.get("RTOW_LAYOUT_INFO")
    os.environ["RTOW_LAYOUT_INFO"] = "1"
    try:
        for gs, side in ((32, 32), (0, 20)):
            capfd.readouterr()
            rtow.Scene.build("final_ned", n=1, image="synthetic", ground_side=gs).check()
            err = capfd.readouterr().err
            assert f"grid {side}x{side}" in err, err[-2000:]
    finally:
        if old is None:
            os.environ.pop("RTOW_LAYOUT_INFO", None)
        else:
            os.environ["RTOW_LAYOUT_INFO"] = old


def test_layout_digest_tool_runs(tmp_path):
    """tools/layout_digest.py's dump path: both trees, deterministic bytes."""
    sc = rtow.Scene.build("final_ned", n=1, image="synthetic")
    a, b = _dump(sc, tmp_path), _dump(sc, tmp_path)
    assert a == b
    assert _dump(sc, tmp_path, "ref") != a
