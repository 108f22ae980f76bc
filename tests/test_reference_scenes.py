"""The reference's non-NED scene builders, randomScene() (scenes.h:29-120) and
cornellBox() (scenes.h:220-353): main.cpp renders the NED builders, but these
are part of the reference's scene API, so rtow_build_scene builds them too
(RTOW_SCENE_RANDOM / RTOW_SCENE_CORNELL, rtow_scene.cpp randomScene /
cornellBox).

Fixtures (tests/golden/make_extra_golden.py): the harness calls the
reference's own functions -- randomScene() in the reference's directory, so it
loads its ./input_images/earth1300x1300.jpg (staged in input_images/ as data),
and in an empty directory, where stbi_load fails and the glass fallback
(scenes.h:104-109) is built; cornellBox() as it is.

CPU: the product's builders give byte-identical scene graphs (same draws,
texels), and the C oracle reproduces the reference's images bit for bit.
GPU: the HIP path within the north-star bar, segment counts equal."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import rtow
import scene_io as sio

MANIFEST = json.load(open(os.path.join(sio.GOLDEN, "manifest_extra.json")))
CASES = {c["name"]: c for c in MANIFEST["cases"]}
EARTH1300 = os.path.join(sio.REPO, "input_images", "earth1300x1300.jpg")
NAMES = ["random_ref", "random_ref_noimg", "cornell_box"]


def _product(name):
    c = CASES[name]
    if c["image"] == "reference":
        return rtow.Scene.build(c["scene"], n=c["n"], image="jpeg", image_path=EARTH1300, scene_seed=1)
    return rtow.Scene.build(c["scene"], n=c["n"], image="none", scene_seed=1)


def _fixture(name):
    """The reference's scene graph with its texels re-attached (the JPEG the
    reference decoded: our decoder is stb_image's, tests/test_jpeg.py)."""
    d = sio.load_scene(os.path.join(sio.GOLDEN, name + ".scn"))
    if CASES[name]["image"] == "reference":
        px = rtow.decode_jpeg(open(EARTH1300, "rb").read())
        d = dict(d)
        d["texels"] = np.ascontiguousarray(px.reshape(-1))
    return d


def test_staged_earth1300():
    """input_images/earth1300x1300.jpg is the reference's file (scenes.h:47),
    and our decoder gives the texels the fixture's reference run loaded."""
    data = open(EARTH1300, "rb").read()
    assert hashlib.sha256(data).hexdigest() == "a08d00d779a2a0e1e139c833193f075cf3daefaef7ac30374df272e22550f1b9"
    px = rtow.decode_jpeg(data)
    assert px.shape == (1300, 1300, 3)
    assert hashlib.sha256(px.tobytes()).hexdigest() == CASES["random_ref"]["texel_sha256"]


@pytest.mark.parametrize("name", NAMES)
def test_scene_graph_byte_identical(name, tmp_path):
    c = CASES[name]
    s = _product(name)
    path = str(tmp_path / "p.scn")
    s.save(path)
    p = sio.load_scene(path)
    g = sio.load_scene(os.path.join(sio.GOLDEN, name + ".scn"))
    assert p["root"] == g["root"]
    for k in ("hitables", "refs", "materials", "textures", "images"):
        assert p[k].tobytes() == g[k].tobytes(), k
    assert p["perlin"].tobytes() == g["perlin"].tobytes()
    assert len(p["texels"]) == c["texel_bytes"]
    assert hashlib.sha256(p["texels"].tobytes()).hexdigest() == c["texel_sha256"]
    assert len(p["hitables"]) == c["n_hitables"]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_bit_exact(name):
    c = CASES[name]
    W, H = c["width"], c["height"]
    arrays = sio.SceneArrays(_fixture(name))
    cam = sio.camera_from_file(os.path.join(sio.GOLDEN, f"cam_{W}x{H}.cam"))
    p = sio.default_params(W, H, c["spp"], seed=c["seed"])
    lin, bgra, cnt = sio.oracle_render(ctypes.addressof(arrays.view), cam, p)
    glin, gbgra = sio.golden_image(name, W, H)
    assert np.array_equal(lin.reshape(H, W, 3).view(np.uint32), glin.view(np.uint32))
    assert np.array_equal(bgra.reshape(H, W, 4), gbgra)
    assert cnt.samples == W * H * c["spp"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("tree", ["sah", "reference"])
def test_gpu_matches_reference(name, tree, gpu_ctx):
    c = CASES[name]
    W, H = c["width"], c["height"]
    scene = _product(name)
    cam = sio.camera_from_file(os.path.join(sio.GOLDEN, f"cam_{W}x{H}.cam"))
    p = rtow.params(W, H, c["spp"], seed=c["seed"])
    ctx = rtow.Context(0)
    try:
        ctx.set_tree(tree)
        ctx.upload(scene)
        _, lin, st = ctx.render(rtow.Camera.from_buffer_copy(bytes(cam)), p)
    finally:
        ctx.close()
    glin, _ = sio.golden_image(name, W, H)
    _, _, oc = sio.oracle_render(scene.view_ptr, cam, sio.RtowParams.from_buffer_copy(bytes(p)))
    g = np.asarray(lin, np.float64).reshape(-1, 3)
    rms = np.sqrt(np.mean((g - glin.reshape(-1, 3).astype(np.float64)) ** 2, axis=0))
    print(f"{name} [{tree}]: rms vs reference {rms} segments gpu {st.segments} oracle {oc.segments}")
    assert (rms <= 1e-4).all(), rms
    assert st.segments == oc.segments
