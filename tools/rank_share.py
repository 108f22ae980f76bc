"""Predicts multi-GPU strong scaling on ONE GPU: renders each rank's tile
share of a frame (world N, rank r) one after another and reports per-rank
kernel time, max over ranks and the implied efficiency
T(1) / (N * max_r T(r)) -- the bench's max-over-ranks clock without RCCL.

  python tools/rank_share.py      RS_SCENE=random_ned|final_ned|cornell|...  RS_W, RS_H, RS_SPP
                                  RS_SPC="0" (0: automatic chunking)  RS_WORLDS="1,2,4,8"
                                  RS_CHECK=K: assemble the largest world's linear slabs into the frame
                                  (rtow_assemble_linear_device) and compare K random pixels with the
                                  C oracle at the same spp (RS_THREADS host threads)

With RS_WORLDS without 1, efficiency is against N x the mean share (the
whole frame is not rendered).
"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
EARTH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "input_images", "1_earth_8k.jpg")  # the benched scenes' texture (scenes.h:140)
sys.path.insert(0, os.path.join(REPO, "ray-tracing-one-weekend_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import rtow  # noqa: E402

SCENE = os.environ.get("RS_SCENE", "random_ned")
DEF = {"random_ned": (1920, 1080, 1024), "final_ned": (4096, 4096, 8192), "cornell": (800, 800, 4096),
       "cornell_smoke": (800, 800, 4096)}[SCENE]
W = int(os.environ.get("RS_W", DEF[0]))
H = int(os.environ.get("RS_H", DEF[1]))
spp = int(os.environ.get("RS_SPP", DEF[2]))
spcs = [int(v) for v in os.environ.get("RS_SPC", "0").split(",")]
worlds = [int(v) for v in os.environ.get("RS_WORLDS", "1,2,4,8").split(",")]
check = int(os.environ.get("RS_CHECK", "0"))
threads = int(os.environ.get("RS_THREADS", "16"))
torch.cuda.init()
scene = rtow.Scene.build(SCENE, n=487 if SCENE == "random_ned" else 1, image="jpeg", image_path=EARTH, scene_seed=1)
cam = rtow.camera_main(W, H)
ctx = rtow.Context(0)
ctx.upload(scene)
print(f"rank_share: {SCENE} {W}x{H}x{spp}, worlds {worlds}, chunking {spcs} (0 = automatic)", flush=True)
wmax = max(worlds)
stride = rtow.rank_tile_count(W, H, 0, min(worlds)) * 64
slab = torch.zeros(stride * 4, dtype=torch.uint8, device="cuda")
ctx.render_tiles_device(cam, rtow.params(W, H, 1, seed=1, rank=0, world=wmax), slab.data_ptr())  # warm
lin = None
for spc in spcs:
    t1 = None
    for world in worlds:
        ms, segs = [], 0
        keep = check and spc == spcs[0] and world == wmax
        if keep:
            sw = rtow.rank_tile_count(W, H, 0, world) * 64
            lin = torch.zeros((world, sw * 3), dtype=torch.float32, device="cuda")
        for r in range(world):
            p = rtow.params(W, H, spp, seed=1, rank=r, world=world, samples_per_chunk=spc)
            pl = rtow.plan(p, ctx)
            st = ctx.render_tiles_device(cam, p, slab.data_ptr(), lin[r].data_ptr() if keep else None)
            ms.append(st.kernel_ms)
            segs += st.segments
            print(f"  world {world} rank {r}: {st.kernel_ms:9.1f} ms  {st.segments / st.kernel_ms / 1e3:8.1f} Mray/s  "
                  f"items of {pl.samples_per_chunk} (n_big {pl.n_big}, tail {pl.tail_samples} in {pl.n_tail})",
                  flush=True)
        mx, mean = max(ms), sum(ms) / len(ms)
        if world == 1:
            t1 = mx
        eff = t1 / (world * mx) if t1 else mean / mx
        print(f"spc {spc:3d} world {world}: rank ms min {min(ms):8.1f} max {mx:8.1f} mean {mean:8.1f} "
              f"sum {sum(ms):8.1f}  max/mean {mx / mean:.4f}  efficiency {eff:.3f}"
              + ("" if t1 else " (vs N x mean share)") + f"  frame Mray/s at max {segs / mx / 1e3:.1f}", flush=True)
if check:
    import scene_io as sio

    world = wmax
    sw = rtow.rank_tile_count(W, H, 0, world) * 64
    frame = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
    ctx.assemble_linear_device(W, H, world, lin.data_ptr(), sw, frame.data_ptr())
    f = frame.cpu().numpy().reshape(-1, 3)
    # every pixel written once: the numpy mirror of the assembly agrees
    ref = rtow.assemble(lin.cpu().numpy().reshape(world, sw, 3), W, H, world).reshape(-1, 3)
    assert np.array_equal(f.view(np.uint32), ref.view(np.uint32)), "assembled frame differs from the slabs"
    rng = np.random.default_rng(5)
    pix = rng.choice(W * H, size=check, replace=False).astype(np.uint32)
    p = rtow.params(W, H, spp, seed=1)
    t0 = time.perf_counter()
    olin, _, oc = sio.oracle_render(scene.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                    sio.RtowParams.from_buffer_copy(bytes(p)), pixels=pix, threads=threads)
    dt = time.perf_counter() - t0
    g = f[pix].astype(np.float64)
    d = np.abs(g - olin).max(axis=1)
    rms = np.sqrt(np.mean((g - olin) ** 2, axis=0))
    print(f"CHECK assembled {world}-rank frame vs oracle, {check} random pixels x {spp} spp ({dt:.1f} s on "
          f"{threads} threads): rms {rms} max|d| {d.max():.3g} pixels>1e-3 {int((d > 1e-3).sum())} "
          f"bit-identical {float(np.mean(d == 0)):.4f} finite {bool(np.isfinite(f).all())}", flush=True)
ctx.close()
