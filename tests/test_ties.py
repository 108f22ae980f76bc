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
