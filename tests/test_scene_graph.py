"""The product's host scene builders (librtow_hip.so, rtow_scene.cpp) build
the SAME world the reference builds: byte-identical flattened scene graph,
Perlin tables, texel hash and random-draw count, for every golden case."""
import hashlib
import os

import numpy as np
import pytest

import rtow
import scene_io as sio

CASES = [c["name"] for c in sio.manifest()["cases"]]


def product_scene(c, tmp_path):
    s = rtow.Scene.build(c["scene"], n=c["n"], image=c["image"], scene_seed=sio.manifest()["scene_seed"])
    path = str(tmp_path / "p.scn")
    s.save(path)
    return s, sio.load_scene(path)


@pytest.mark.parametrize("name", CASES)
def test_scene_graph_byte_identical(name, tmp_path):
    c = sio.golden_case(name)
    s, p = product_scene(c, tmp_path)
    g = sio.load_scene(os.path.join(sio.GOLDEN, name + ".scn"))
    assert p["root"] == g["root"]
    for k in ("hitables", "refs", "materials", "textures", "images"):
        assert p[k].tobytes() == g[k].tobytes(), k
    assert p["perlin"].tobytes() == g["perlin"].tobytes()
    assert len(p["texels"]) == c["texel_bytes"]
    if c["texel_bytes"]:
        assert hashlib.sha256(p["texels"].tobytes()).hexdigest() == c["texel_sha256"]
    assert s.draws == c["scene_draws"]


@pytest.mark.parametrize("W,H", [(200, 100), (64, 36), (48, 48), (37, 23)])
def test_camera_matches_reference(W, H):
    cam = rtow.camera_main(W, H)
    assert bytes(cam) == open(os.path.join(sio.GOLDEN, f"cam_{W}x{H}.cam"), "rb").read()


def test_save_load_roundtrip(tmp_path):
    s = rtow.Scene.build("cornell_smoke")
    a = str(tmp_path / "a.scn")
    b = str(tmp_path / "b.scn")
    s.save(a)
    rtow.Scene.load(a).save(b)
    assert open(a, "rb").read() == open(b, "rb").read()


def test_synthetic_image_formula():
    assert np.array_equal(rtow.synthetic_image(2048, 1024), sio.synthetic_image(2048, 1024))
    assert np.array_equal(rtow.synthetic_image(7, 3), sio.synthetic_image(7, 3))


def test_scene_check_bounds():
    # random scene: root Translate + BVH; cornell: lists, boxes, instances, a medium
    st, ch = rtow.Scene.build("random_ned", n=487).check()
    assert 9 <= st <= 16 and ch == 1
    st, ch = rtow.Scene.build("cornell_smoke").check()
    assert st <= 64 and ch == 3  # Translate(root) > Translate > RotateY; FlipNormals folds into its rectangle


def test_medium_under_bvh_rejected(tmp_path):
    """A ConstantMedium below a BvhNode draws random numbers in the
    reference's exhaustive visit order; the device path refuses it loudly."""
    s = rtow.Scene.build("random_ned", n=100)
    d = sio.load_scene(_save(s, tmp_path))
    h = d["hitables"]
    idx = int(np.nonzero(h["kind"] == 1)[0][-1])  # some sphere under the BVH
    med = np.zeros(1, sio.HITABLE)
    med[0]["kind"] = 12
    med[0]["a"] = idx
    med[0]["b"] = 0
    med[0]["f"][0] = 0.5
    d["hitables"] = np.concatenate([h, med])
    # re-point a BVH child at the medium
    bvh = int(np.nonzero(d["hitables"]["kind"] == 11)[0][-1])
    d["hitables"][bvh]["a"] = len(h)
    arr = sio.SceneArrays(d)
    import ctypes

    rc = rtow.lib().rtow_scene_check(ctypes.addressof(arr.view), None, None)
    assert rc == rtow.E_UNSUPPORTED
    assert b"BvhNode" in rtow.lib().rtow_last_error()


def _save(s, tmp_path):
    p = str(tmp_path / "s.scn")
    s.save(p)
    return p
