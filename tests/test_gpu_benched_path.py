"""Parity on the exact path bench.py times ("Pin parity on the
benched path").

The bench renders config 2 at 1920x1080x1024 spp through
rtow_render_tiles_device (rank 0 of 1) with automatic chunking: 128-sample work
items (seven per pixel) and a halving tail of 64/32/16/8/4/2/1/1 samples, each
chunk summed in float in sample order (main.cpp:939-946) and added to the
pixel's fixed-point sum.  Config 5 is quoted for 8 GPUs; one rank's share of
its 4096x4096 frame also runs on 128-sample items.  These tests render those
exact launches and compare a random pixel sample with the C oracle (the
reference's recursion, main.cpp:939-955 / color.h:12-59) at the same spp.

The bench renders configs 2 and 5 with the reference's own earth texture
(input_images/1_earth_8k.jpg, scenes.h:140), so these tests do too, and add to
the random sample pixels whose paths see the earth (found by rendering the
slab at 2 spp with the synthetic stand-in and with the JPEG and taking the
pixels that differ).

Bar: per-channel RMS <= 1e-4 (BASELINE north_star) and at most 1 pixel per
10^5 off by more than 1e-3.
"""
import os

import numpy as np
import pytest

import rtow
import scene_io as sio

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-4
EARTH = os.path.join(sio.REPO, "input_images", "1_earth_8k.jpg")


def _earth_scene(name, n):
    return rtow.Scene.build(name, n=n, image="jpeg", image_path=EARTH, scene_seed=1)


def _earth_positions(ctx, name, n, W, H, rank, world, k, seed):
    """Up to k slab positions whose 2-spp values change when the synthetic
    texture is replaced by the earth JPEG: pixels whose paths see the earth."""
    lins = []
    for sc in (rtow.Scene.build(name, n=n, image="synthetic", scene_seed=1), _earth_scene(name, n)):
        lins.append(_slab_render(ctx, sc, W, H, 2, 7, rank, world)[3])
    idx = rtow.rank_pixels(W, H, rank, world)
    hit = np.flatnonzero((idx >= 0) & (lins[0] != lins[1]).any(axis=1))
    assert hit.size >= k, hit.size
    return np.random.default_rng(seed).choice(hit, size=k, replace=False)


def _slab_render(ctx, scene, W, H, spp, seed, rank, world):
    """One rtow_render_tiles_device launch (bench.py's HipRank.step) with a
    linear slab; returns (linear frame values of the rank's pixels keyed by
    framebuffer index, stats, plan)."""
    import torch

    ctx.upload(scene)
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=seed, rank=rank, world=world)
    stride = rtow.rank_tile_count(W, H, rank, world) * 64
    bgra = torch.zeros(stride * 4, dtype=torch.uint8, device="cuda")
    lin = torch.zeros(stride * 3, dtype=torch.float32, device="cuda")
    st = ctx.render_tiles_device(cam, p, bgra.data_ptr(), lin.data_ptr())
    torch.cuda.synchronize()
    idx = rtow.rank_pixels(W, H, rank, world)
    return cam, p, idx, lin.cpu().numpy().reshape(-1, 3), st, rtow.plan(p, ctx)


def _compare(scene, cam, p, idx, lin, n_pix, seed, extra=None):
    ok = np.flatnonzero(idx >= 0)
    rng = np.random.default_rng(seed)
    pick = rng.choice(ok, size=n_pix, replace=False)
    if extra is not None:
        pick = np.union1d(pick, extra)
    pix = idx[pick].astype(np.uint32)
    olin, _, oc = sio.oracle_render(scene.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                    sio.RtowParams.from_buffer_copy(bytes(p)), pixels=pix, threads=16)
    g = lin[pick].astype(np.float64)
    d = np.abs(g - olin).max(axis=1)
    rms = np.sqrt(np.mean((g - olin) ** 2, axis=0))
    return rms, d, oc


def test_config2_bench_frame_1024spp(gpu_ctx):
    """Config 2 exactly as benched: randomScene_NED n=487 with the earth
    texture, 1920x1080x1024, seed 1, one rank, automatic chunking (128-sample
    items, n_big 7, a 128-sample halving tail in 8 chunks); 3000 random
    pixels and 500 that see the earth vs the oracle."""
    W, H, spp = 1920, 1080, 1024
    earth = _earth_positions(gpu_ctx, "random_ned", 487, W, H, 0, 1, 500, 5)
    scene = _earth_scene("random_ned", 487)
    cam, p, idx, lin, st, pl = _slab_render(gpu_ctx, scene, W, H, spp, 1, 0, 1)
    assert (pl.samples_per_chunk, pl.n_big, pl.tail_samples, pl.n_tail) == (128, 7, 128, 8), pl.as_dict()
    assert st.samples == W * H * spp
    rms, d, oc = _compare(scene, cam, p, idx, lin, 3000, 0, extra=earth)
    n_off = int((d > 1e-3).sum())
    print(f"BENCHED config2 1920x1080x1024 (earth JPEG): plan {pl.as_dict()} rms {rms} max|d| {d.max():.3g} "
          f"pixels>1e-3 {n_off}/{d.size} bit-identical {float(np.mean(d == 0)):.4f} "
          f"rays/sample gpu {st.segments / st.samples:.4f} oracle-sample {oc.segments / oc.samples:.4f} "
          f"kernel {st.kernel_ms:.1f} ms")
    assert np.isfinite(lin).all()
    assert (rms <= RMS_TOL).all(), rms
    assert n_off <= int(1e-5 * d.size)


def test_config2_eight_gpu_shares_1024spp(gpu_ctx):
    """The launches an 8-GPU run of config 2 times: bench.py
    at N > 1 plans every rank's share by itself (no RTOW_FLAG_FRAME_PLAN), so
    each of the eight ranks cuts 32-sample items (n_big 31, a 32-sample halving
    tail in 6 chunks) and sums them in float in sample order (main.cpp:939-946).
    All eight shares of 1920x1080x1024 (earth JPEG, seed 1) are rendered with
    rtow_render_tiles_device, assembled with rtow_assemble_linear_device (the
    tile interleave standing for main.cpp:936's column interleave), and 2000
    random pixels plus 300 that see the earth are compared with the oracle at
    1024 spp.  The shares' segments must sum to the one-rank render's.  Rank 0
    of world 4 (64-sample items, n_big 15, tail in 7) is checked the same way
    on 1000 pixels of its slab."""
    import torch

    W, H, spp, world = 1920, 1080, 1024, 8
    earth_pos = _earth_positions(gpu_ctx, "random_ned", 487, W, H, 0, 1, 300, 8)
    earth = rtow.rank_pixels(W, H, 0, 1)[earth_pos]
    scene = _earth_scene("random_ned", 487)
    gpu_ctx.upload(scene)
    cam = rtow.camera_main(W, H)
    stride = rtow.rank_tile_count(W, H, 0, world) * 64
    bgra = torch.zeros((world, stride * 4), dtype=torch.uint8, device="cuda")
    lin = torch.zeros((world, stride * 3), dtype=torch.float32, device="cuda")
    segs, ms = 0, []
    for r in range(world):
        p = rtow.params(W, H, spp, seed=1, rank=r, world=world)
        pl = rtow.plan(p, gpu_ctx)
        assert (pl.samples_per_chunk, pl.n_big, pl.tail_samples, pl.n_tail) == (32, 31, 32, 6), (r, pl.as_dict())
        st = gpu_ctx.render_tiles_device(cam, p, bgra[r].data_ptr(), lin[r].data_ptr())
        torch.cuda.synchronize()
        segs += st.segments
        ms.append(st.kernel_ms)
    fl = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
    gpu_ctx.assemble_linear_device(W, H, world, lin.data_ptr(), stride, fl.data_ptr())
    torch.cuda.synchronize()
    frame = fl.cpu().numpy().reshape(-1, 3)
    # the whole frame as one rank renders it: same paths, so the same segments
    st1 = _slab_render(gpu_ctx, scene, W, H, spp, 1, 0, 1)[4]
    assert segs == st1.segments, (segs, st1.segments)
    pick = np.union1d(np.random.default_rng(10).choice(W * H, size=2000, replace=False), earth)
    p1 = rtow.params(W, H, spp, seed=1)
    olin, _, oc = sio.oracle_render(scene.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                    sio.RtowParams.from_buffer_copy(bytes(p1)), pixels=pick.astype(np.uint32),
                                    threads=16)
    g = frame[pick].astype(np.float64)
    d = np.abs(g - olin).max(axis=1)
    rms = np.sqrt(np.mean((g - olin) ** 2, axis=0))
    n_off = int((d > 1e-3).sum())
    # rank 0 of world 4
    cam4, p4, idx4, lin4, st4, pl4 = _slab_render(gpu_ctx, scene, W, H, spp, 1, 0, 4)
    assert (pl4.samples_per_chunk, pl4.n_big, pl4.tail_samples, pl4.n_tail) == (64, 15, 64, 7), pl4.as_dict()
    rms4, d4, _ = _compare(scene, cam4, p4, idx4, lin4, 1000, 11)
    print(f"BENCHED config2 8 shares 1920x1080x1024 (per-rank plan 32/31/32/6): share kernel ms "
          f"{min(ms):.1f}..{max(ms):.1f}; rms {rms} max|d| {d.max():.3g} pixels>1e-3 {n_off}/{d.size} "
          f"bit-identical {float(np.mean(d == 0)):.4f}; segments 8 shares {segs} = 1 rank {st1.segments}; "
          f"world-4 rank 0 (64/15/64/7): rms {rms4} max|d| {d4.max():.3g}")
    assert np.isfinite(frame).all()
    assert (rms <= RMS_TOL).all(), rms
    assert n_off <= 1
    assert (rms4 <= RMS_TOL).all(), rms4
    assert int((d4 > 1e-3).sum()) <= 1


def test_config5_rank_share_128_sample_items(gpu_ctx):
    """Config 5's 8-GPU split: rank 0's share of final_ned 4096x4096 at 512 spp,
    which picks 128-sample items (n_big 3 + the 128-sample tail) as the 8192-spp
    bench share does (n_big 63), with the earth texture; 500 random pixels of
    the slab and 200 that see the earth vs the oracle."""
    W, H, spp = 4096, 4096, 512
    earth = _earth_positions(gpu_ctx, "final_ned", 1, W, H, 0, 8, 200, 6)
    scene = _earth_scene("final_ned", 1)
    cam, p, idx, lin, st, pl = _slab_render(gpu_ctx, scene, W, H, spp, 1, 0, 8)
    assert (pl.samples_per_chunk, pl.n_big, pl.tail_samples, pl.n_tail) == (128, 3, 128, 8), pl.as_dict()
    full = rtow.plan(rtow.params(W, H, 8192, rank=0, world=8), gpu_ctx)
    assert (full.samples_per_chunk, full.n_big, full.n_tail) == (128, 63, 8)
    rms, d, oc = _compare(scene, cam, p, idx, lin, 500, 1, extra=earth)
    n_off = int((d > 1e-3).sum())
    print(f"BENCHED config5 share 0/8 4096^2x512 (earth JPEG): plan {pl.as_dict()} rms {rms} max|d| {d.max():.3g} "
          f"pixels>1e-3 {n_off}/{d.size} bit-identical {float(np.mean(d == 0)):.4f} kernel {st.kernel_ms:.1f} ms")
    assert np.isfinite(lin).all()
    assert (rms <= RMS_TOL).all(), rms
    assert n_off <= int(1e-5 * d.size)


@pytest.mark.parametrize("scene", ["cornell", "cornell_smoke"])
def test_configs_3_4_bench_frame_4096spp(scene, gpu_ctx):
    """Configs 3 and 4 exactly as benched: 800x800x4096,
    one rank, automatic chunking -- 128-sample items, n_big 31, a 128-sample
    halving tail in 8 chunks, each chunk's samples summed in float in sample
    order (main.cpp:939-955) through MODE 5's top-level scan (hitableList.h:
    20-38) and, for cornell_smoke, the medium (constantMedium.h:26-74).  1000
    random pixels of the frame vs the oracle at 4096 spp; then 8 random whole
    tiles rendered alone (rank t of world = the frame's tile count, with
    RTOW_FLAG_FRAME_PLAN: the bench's chunks) must give the frame's values bit
    for bit and the oracle's segment count on those 512 pixels exactly."""
    import torch

    W, H, spp = 800, 800, 4096
    sc = rtow.Scene.build(scene, n=1, image="none", scene_seed=1)
    cam, p, idx, lin, st, pl = _slab_render(gpu_ctx, sc, W, H, spp, 1, 0, 1)
    assert (pl.samples_per_chunk, pl.n_big, pl.tail_samples, pl.n_tail) == (128, 31, 128, 8), pl.as_dict()
    assert st.samples == W * H * spp
    rms, d, oc = _compare(sc, cam, p, idx, lin, 1000, 3)
    n_off = int((d > 1e-3).sum())
    frame = np.zeros((W * H, 3), np.float32)
    ok = idx >= 0
    frame[idx[ok]] = lin[ok]
    # whole tiles alone: the segment count of 512 pixels, and the same values
    n_tiles = rtow.tile_count(W, H)
    tiles = np.random.default_rng(4).choice(n_tiles, size=8, replace=False)
    segs, pix, vals = 0, [], []
    bgra = torch.zeros(64 * 4, dtype=torch.uint8, device="cuda")
    tl = torch.zeros(64 * 3, dtype=torch.float32, device="cuda")
    for t in tiles:
        q = rtow.params(W, H, spp, seed=1, rank=int(t), world=n_tiles, flags=rtow.FLAG_FRAME_PLAN)
        qs = gpu_ctx.render_tiles_device(cam, q, bgra.data_ptr(), tl.data_ptr())
        torch.cuda.synchronize()
        ti = rtow.rank_pixels(W, H, int(t), n_tiles)
        assert (ti >= 0).all() and qs.pixels == 64
        segs += qs.segments
        pix.append(ti)
        vals.append(tl.cpu().numpy().reshape(64, 3))
    pix, vals = np.concatenate(pix), np.concatenate(vals)
    assert np.array_equal(vals.view(np.uint32), frame[pix].view(np.uint32))
    _, _, tc = sio.oracle_render(sc.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                 sio.RtowParams.from_buffer_copy(bytes(p)), pixels=pix.astype(np.uint32), threads=16)
    print(f"BENCHED {scene} 800x800x4096: plan {pl.as_dict()} rms {rms} max|d| {d.max():.3g} pixels>1e-3 "
          f"{n_off}/1000 bit-identical {float(np.mean(d == 0)):.4f} rays/sample gpu {st.segments / st.samples:.4f} "
          f"oracle-sample {oc.segments / oc.samples:.4f}; 8 tiles: segments gpu {segs} oracle {tc.segments} "
          f"kernel {st.kernel_ms:.1f} ms")
    assert np.isfinite(lin).all()
    assert (rms <= RMS_TOL).all(), rms
    assert d.max() <= 1e-3
    assert segs == tc.segments
