"""Predicts multi-GPU strong scaling on ONE GPU: renders each rank's tile
share of the bench frame (world N, rank r) one after another and reports
per-rank kernel time, max over ranks and the implied efficiency
T(1) / (N * max_r T(r)) -- the bench's max-over-ranks clock without RCCL.

  python tools/rank_share.py            (RS_SPP, RS_SPC="64,16", RS_WORLDS="1,2,4,8")
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-one-weekend_amd"))
import rtow  # noqa: E402

W, H = 1920, 1080
spp = int(os.environ.get("RS_SPP", "1024"))
spcs = [int(v) for v in os.environ.get("RS_SPC", "64,16").split(",")]
worlds = [int(v) for v in os.environ.get("RS_WORLDS", "1,2,4,8").split(",")]
torch.cuda.init()
scene = rtow.Scene.build("random_ned", n=487, image="synthetic", scene_seed=1)
cam = rtow.camera_main(W, H)
ctx = rtow.Context(0)
ctx.upload(scene)
slab = torch.zeros(rtow.rank_tile_count(W, H, 0, 1) * 64 * 4, dtype=torch.uint8, device="cuda")
ctx.render_tiles_device(cam, rtow.params(W, H, 64, seed=1), slab.data_ptr())  # warm
for spc in spcs:
    t1 = None
    for world in worlds:
        ms = []
        for r in range(world):
            p = rtow.params(W, H, spp, seed=1, rank=r, world=world, samples_per_chunk=spc)
            st = ctx.render_tiles_device(cam, p, slab.data_ptr())
            ms.append(st.kernel_ms)
        mx = max(ms)
        if world == 1:
            t1 = mx
        eff = t1 / (world * mx) if t1 else float("nan")
        print(f"spc {spc:3d} world {world}: rank ms min {min(ms):8.1f} max {mx:8.1f} sum {sum(ms):8.1f}  "
              f"efficiency {eff:.3f}", flush=True)
ctx.close()
