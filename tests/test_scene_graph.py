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


def _medium_under_bvh(tmp_path, behind_translate):
    s = rtow.Scene.build("random_ned", n=100)
    d = sio.load_scene(_save(s, tmp_path))
    h = d["hitables"]
    idx = int(np.nonzero(h["kind"] == 1)[0][-1])  # some sphere under the BVH
    extra = np.zeros(3 if behind_translate else 2, sio.HITABLE)
    extra[0] = h[idx]  # the boundary: a copy of that sphere
    extra[1]["kind"] = 12  # ConstantMedium(sphere, density 0.5, phase material 0)
    extra[1]["a"] = len(h)
    extra[1]["b"] = 0
    extra[1]["f"][0] = 0.5
    target = len(h) + 1
    if behind_translate:
        extra[2]["kind"] = sio.HIT_TRANSLATE
        extra[2]["a"] = len(h) + 1
        extra[2]["f"][:3] = (0.0, 1.0, 0.0)
        target = len(h) + 2
    d["hitables"] = np.concatenate([h, extra])
    bvh = int(np.nonzero(d["hitables"]["kind"] == 11)[0][-1])  # re-point a BVH child
    d["hitables"][bvh]["a"] = target
    return sio.SceneArrays(d)


def test_medium_under_bvh_accepted(tmp_path):
    """A ConstantMedium below a BvhNode is replayed in the reference's
    exhaustive visit order (DProg; GPU parity: tests/test_medium_bvh.py)."""
    import ctypes

    arr = _medium_under_bvh(tmp_path, False)
    assert rtow.lib().rtow_scene_check(ctypes.addressof(arr.view), None, None) == rtow.OK


def test_medium_under_bvh_behind_instance_accepted(tmp_path):
    """...and behind an instance or list there too: no program replays the
    interval and frame such a medium sees, so the world goes to the
    exact-order kernel (MODE 6, xhit; GPU parity: tests/test_medium_exact.py)."""
    import ctypes

    arr = _medium_under_bvh(tmp_path, True)
    assert rtow.lib().rtow_scene_check(ctypes.addressof(arr.view), None, None) == rtow.OK


def _save(s, tmp_path):
    p = str(tmp_path / "s.scn")
    s.save(p)
    return p


@pytest.mark.parametrize("grid,dtree,expect", [("1", "1", [1, 2, 7, 3, 3, 2, 5]),
                                               ("0", "1", [6, 3, 3, 2, 2, 5]), ("0", "0", [0, 3, 3, 2, 2, 5])])
def test_final_scene_top_level_items(grid, dtree, expect):
    """final_ned's top-level scan (buildTop, printed by RTOW_LAYOUT_INFO).  By
    default the ground's 20 x 20 Boxes are a grid (TOP_GRID = 7, walked by
    MODE 8) and the rest of their run -- the light (a rectangle, 1) and four
    spheres (2, one item: a grid world scans a run of spheres in one frame as
    one item) -- is scanned in place; with RTOW_GRID=0 the first tree (ground
    Boxes, light, spheres) runs in trace_dnodes' loop with leaf slots
    (TOP_DTREE = 6) unless RTOW_DTREE=0 sends it to the general traversal
    (TOP_GENERIC = 0); then two media (3), two spheres (2; one run item in the
    grid world), the cloud (5)."""
    import subprocess
    import sys
    code = ("import rtow; rtow.Scene.build('final_ned', n=100, image='synthetic').check()")
    env = dict(os.environ, RTOW_LAYOUT_INFO="1", RTOW_DTREE=dtree, RTOW_GRID=grid)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True,
                         cwd=os.path.dirname(rtow.__file__)).stderr
    kinds = [int(l.split(" kind ")[1].split()[0]) for l in out.splitlines() if l.startswith("rtow-layout: top[")]
    assert kinds == expect
