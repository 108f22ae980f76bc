"""ConstantMedium below a BvhNode.  The reference visits BOTH children of every
BvhNode whose own box the ray hits, with the interval the node received
(bvhNode.h:66-96), so a medium there draws its numbers (constantMedium.h:26-74:
one per call, a second when the ray crosses its boundary) whenever its
ancestors' boxes pass AABB::hit (aabb.h:22-43), in depth-first left-to-right
order, and an n == 1 node calls its one leaf twice (bvhNode.h:38-39).

Fixture: tests/golden/make_extra_golden.py `medium_bvh` (ref_harness.cpp
mediumBvhNed: the reference's own classes; four media in the BVH, one of them
the leaf of an n == 1 node, box and sphere boundaries).  CPU: the oracle
bit-exact against it.  GPU: the HIP path within the north-star bar, segment
count equal to the oracle's."""
import ctypes
import json
import os

import numpy as np
import pytest

import rtow
import scene_io as sio

MANIFEST = json.load(open(os.path.join(sio.GOLDEN, "manifest_extra.json")))
CASE = {c["name"]: c for c in MANIFEST["cases"]}["medium_bvh"]


def _setup():
    c = CASE
    W, H = c["width"], c["height"]
    scene = sio.load_scene(os.path.join(sio.GOLDEN, "medium_bvh.scn"))
    cam = sio.camera_from_file(os.path.join(sio.GOLDEN, f"cam_{W}x{H}.cam"))
    p = sio.default_params(W, H, c["spp"], seed=c["seed"])
    return scene, sio.SceneArrays(scene), cam, p


def test_scene_has_media_below_bvh_and_an_n1_medium():
    d, _, _, _ = _setup()
    h = d["hitables"]
    bvh = np.nonzero(h["kind"] == sio.HIT_BVH_NODE)[0]
    kids = {int(h[i]["a"]) for i in bvh} | {int(h[i]["b"]) for i in bvh}
    media = {int(i) for i in np.nonzero(h["kind"] == 12)[0]}  # RTOW_HIT_CONSTANT_MEDIUM
    assert len(media & kids) == 4
    assert any(int(h[i]["a"]) == int(h[i]["b"]) and int(h[i]["a"]) in media for i in bvh)


def test_oracle_medium_bvh_matches_reference_bit_exact():
    c = CASE
    W, H = c["width"], c["height"]
    _, arrays, cam, p = _setup()
    lin, bgra, cnt = sio.oracle_render(ctypes.addressof(arrays.view), cam, p)
    glin, gbgra = sio.golden_image("medium_bvh", W, H)
    assert np.array_equal(lin.reshape(H, W, 3).view(np.uint32), glin.view(np.uint32))
    assert np.array_equal(bgra.reshape(H, W, 4), gbgra)
    assert cnt.medium_calls > 0


@pytest.mark.gpu
@pytest.mark.parametrize("tree", ["sah", "reference"])
def test_gpu_medium_bvh_matches_reference(gpu_ctx, tree):
    c = CASE
    W, H = c["width"], c["height"]
    d, arrays, ocam, op = _setup()
    gpu_ctx.set_tree(tree)
    try:
        gpu_ctx.upload(sio.ArrayScene(d))
        bgra, lin, st = gpu_ctx.render(rtow.camera_main(W, H), rtow.params(W, H, c["spp"], seed=c["seed"]))
    finally:
        gpu_ctx.set_tree("sah")
    glin, gbgra = sio.golden_image("medium_bvh", W, H)
    a = np.asarray(lin, np.float64).reshape(-1, 3)
    rms = np.sqrt(np.mean((a - glin.reshape(-1, 3)) ** 2, axis=0))
    exact = float(np.mean(lin.reshape(glin.shape) == glin))
    print(f"MEDIUM_BVH rms {rms} exact {exact:.4f}")
    assert (rms <= 1e-4).all(), rms
    assert np.mean(bgra != gbgra) < 0.01
    _, _, cnt = sio.oracle_render(ctypes.addressof(arrays.view), ocam, op)
    assert st.segments == cnt.segments


def _medium_list_boundary_world():
    """BvhNode(ConstantMedium(boundary = HitableList[A, B]), Sphere S): the
    medium's boundary needs the nested general traversal, below a BvhNode."""
    d = sio.scene_dict(rtow.Scene.build("random_ned", n=4, image="none"))  # textures + Perlin tables
    h = np.zeros(6, sio.HITABLE)
    h[0]["kind"], h[0]["a"], h[0]["b"] = sio.HIT_BVH_NODE, 1, 2
    h[0]["f"][:6] = [1, -3, -3, 4, 3, 3]  # the main camera sits at the origin looking along +x
    h[1]["kind"], h[1]["a"], h[1]["b"] = 12, 3, 1  # RTOW_HIT_CONSTANT_MEDIUM: boundary, phase material
    h[1]["f"][0] = 2.0
    h[2]["kind"], h[2]["a"] = sio.HIT_SPHERE, 0
    h[2]["f"][:4] = [2.5, 0, 1.0, 0.5]
    h[3]["kind"], h[3]["a"], h[3]["b"] = sio.HIT_LIST, 0, 2
    for k, c in ((4, -1.0), (5, 1.0)):
        h[k]["kind"], h[k]["a"] = sio.HIT_SPHERE, 0
        h[k]["f"][:4] = [2.5, c, 0, 0.8]
    d["hitables"], d["root"] = h, 0
    d["refs"] = np.array([4, 5], np.uint32)
    m = np.zeros(2, sio.MATERIAL)
    m[0]["kind"], m[0]["texture"] = 1, 0  # Lambertian
    m[1]["kind"], m[1]["texture"] = 5, 0  # Isotropic
    d["materials"] = m
    return d


def test_stack_need_counts_the_continuation_of_a_medium_item():
    """Every DProg item -- a medium too -- runs below the two-entry
    continuation (tin, DK_PROGNEXT) the kernel pushes, so the medium item
    needs 2 + its boundary's 1 (the list's DK_LISTNEXT) = 3 entries."""
    d = _medium_list_boundary_world()
    world = sio.ArrayScene(d)
    sn, _ = sio.scene_check(world)
    assert sn == 3, sn


@pytest.mark.gpu
def test_gpu_medium_with_list_boundary_below_bvh(gpu_ctx):
    d = _medium_list_boundary_world()
    W, H, spp = 32, 24, 16
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=4)
    world = sio.ArrayScene(d)  # keeps the arrays alive while their pointers are used
    gpu_ctx.upload(world)
    _, lin, st = gpu_ctx.render(cam, p)
    olin, _, cnt = sio.oracle_render(world.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                     sio.RtowParams.from_buffer_copy(bytes(p)))
    assert cnt.medium_calls > 0
    assert st.segments == cnt.segments
    assert sio.rms(lin.reshape(-1, 3), olin) <= 1e-4
