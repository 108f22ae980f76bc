"""Exact ties between two leaves (two identical spheres in the random scene).

BvhNode::hit (bvhNode.h:66-96) merges its children's records with
`left.t < right.t ? left : right`, so an exact tie goes to the right subtree
and, over the whole tree, to the LAST tied leaf in left-to-right order.  The
device traverses its own (SAH) tree in its own order and settles ties by the
reference's leaf order instead (rtow_device.hip sph_closer / rebuildSah); these
tests pin that on the oracle (CPU) and on the GPU.
"""
import numpy as np
import pytest

import rtow
import scene_io as sio

W, H, SPP = 64, 36, 4


def _copy(d):
    return {k: (v.copy() if hasattr(v, "copy") else v) for k, v in d.items()}


def _oracle(d, seed=3):
    cam = sio.RtowCamera.from_buffer_copy(bytes(rtow.camera_main(W, H)))
    p = sio.RtowParams.from_buffer_copy(bytes(rtow.params(W, H, SPP, seed=seed)))
    sc = sio.ArrayScene(d)  # keeps the arrays alive while the oracle reads them
    return sio.oracle_render(sc.view_ptr, cam, p)[0]


def _swap_material(d, leaf, other):
    e = _copy(d)
    e["hitables"][leaf]["a"] = d["hitables"][other]["a"]
    return e


def test_oracle_tie_goes_to_later_leaf():
    d, early, late = sio.tie_scene()
    h = d["hitables"]
    assert (h[early]["f"][:4] == h[late]["f"][:4]).all()
    assert h[early]["a"] != h[late]["a"]
    base = _oracle(d)
    # the earlier duplicate never wins: its material cannot show
    assert np.array_equal(_oracle(_swap_material(d, early, late)), base)
    # the later one is on screen and wins
    assert int((np.abs(_oracle(_swap_material(d, late, early)) - base).max(axis=1) > 0).sum()) > 5


@pytest.mark.gpu
def test_gpu_tie_matches_reference_rule(gpu_ctx):
    d, early, late = sio.tie_scene()
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, SPP, seed=3)
    imgs = []
    for dd in (d, _swap_material(d, early, late), _swap_material(d, late, early)):
        sc = sio.ArrayScene(dd)
        gpu_ctx.upload(sc)
        imgs.append(gpu_ctx.render(cam, p)[1].reshape(-1, 3))
    base, early_swapped, late_swapped = imgs
    assert np.array_equal(early_swapped, base)
    assert int((np.abs(late_swapped - base).max(axis=1) > 0).sum()) > 5
    olin = _oracle(d)
    rms = np.sqrt(np.mean((base.astype(np.float64) - olin) ** 2, axis=0))
    assert (rms <= 1e-4).all(), rms


# ---- HitableList ties (hitableList.h:20-38): items scan in order with tmax =
# the closest so far, so a later RECTANGLE (closed interval, xy_rect.h:25)
# takes an exact tie and a later SPHERE (open interval) does not.

def _append_texture_material(d, albedo):
    tex = np.zeros(1, dtype=sio.TEXTURE)
    tex[0]["kind"] = 1  # RTOW_TEX_CONSTANT
    tex[0]["f"][:3] = albedo
    mat = d["materials"][:1].copy()
    mat[0]["kind"] = 1  # RTOW_MAT_LAMBERTIAN
    mat[0]["texture"] = len(d["textures"])
    d["textures"] = np.concatenate([d["textures"], tex])
    d["materials"] = np.concatenate([d["materials"], mat])
    return len(d["materials"]) - 1


def _clone(d, idx, mat):
    """Copy the instance chain / leaf at hitable idx, the leaf with material `mat`."""
    h = d["hitables"]
    e = h[idx:idx + 1].copy()
    if e[0]["kind"] in (6, 7, 8):  # FlipNormals / Translate / RotateY: clone the child first
        e[0]["a"] = _clone(d, int(h[idx]["a"]), mat)
    else:
        e[0]["a"] = mat
    d["hitables"] = np.concatenate([d["hitables"], e])
    return len(d["hitables"]) - 1


def _cornell_with_duplicate(item_kind):
    """cornell with a copy of its first top-level item whose leaf is a
    rectangle (item_kind 'rect') or sphere ('sphere'), in a new colour,
    appended at the END of the root list."""
    d = sio.scene_dict(rtow.Scene.build("cornell"))
    h = d["hitables"]
    lst = int(h[d["root"]]["a"])
    first, count = int(h[lst]["a"]), int(h[lst]["b"])
    items = [int(r) for r in d["refs"][first:first + count]]

    def leaf(i):
        while h[i]["kind"] in (6, 7, 8):
            i = int(h[i]["a"])
        return int(h[i]["kind"])

    want = (3, 4, 5) if item_kind == "rect" else (1,)
    src = next(i for i in items if leaf(i) in want)
    mat = _append_texture_material(d, (0.1, 0.9, 0.9))
    dup = _clone(d, src, mat)
    d["refs"] = np.concatenate([d["refs"], np.array(items + [dup], np.uint32)])
    d["hitables"][lst]["a"] = first = len(d["refs"]) - count - 1
    d["hitables"][lst]["b"] = count + 1
    return d


def test_oracle_list_tie_rule():
    base = _oracle(sio.scene_dict(rtow.Scene.build("cornell")))
    rect_dup = _oracle(_cornell_with_duplicate("rect"))
    sphere_dup = _oracle(_cornell_with_duplicate("sphere"))
    # the later rectangle takes the tie: its new colour shows
    assert int((np.abs(rect_dup - base).max(axis=1) > 0).sum()) > 20
    # the later sphere does not: nothing changes
    assert np.array_equal(sphere_dup, base)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["rect", "sphere"])
def test_gpu_list_ties_match_oracle(kind, gpu_ctx):
    d = _cornell_with_duplicate(kind)
    sc = sio.ArrayScene(d)
    gpu_ctx.upload(sc)
    lin = gpu_ctx.render(rtow.camera_main(W, H), rtow.params(W, H, SPP, seed=3))[1].reshape(-1, 3)
    olin = _oracle(d)
    rms = np.sqrt(np.mean((lin.astype(np.float64) - olin) ** 2, axis=0))
    assert (rms <= 1e-4).all(), rms
    assert float(np.mean(lin == olin)) > 0.5  # most channel values bit-identical (the rest: last-bit product order)
