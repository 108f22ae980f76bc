"""Kernel time of rank 0's share of the config-2 frame against spp, at 1 and
8 ranks and max_depth 50 / 8 / 2 (earth JPEG): the intercept of the last
three points is the launch's fixed cost -- at 8 ranks the drain of the
last items and paths (tools/drain_emulate.py).  python tools/launch_cost_ranks.py"""
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "ray-tracing-one-weekend_amd"))
import rtow  # noqa: E402

W, H = 1920, 1080
torch.cuda.init()
scene = rtow.Scene.build("random_ned", n=487, image="jpeg", image_path=os.path.join(REPO, "input_images", "1_earth_8k.jpg"),
                         scene_seed=1)
cam = rtow.camera_main(W, H)
ctx = rtow.Context(0)
ctx.upload(scene)
slab = torch.zeros(rtow.rank_tile_count(W, H, 0, 1) * 64 * 4, dtype=torch.uint8, device="cuda")
ctx.render_tiles_device(cam, rtow.params(W, H, 1, seed=1), slab.data_ptr())
for world in (1, 8):
    for depth in (50, 8, 2):
        xs, ys = [], []
        for spp in (1, 4, 16, 64, 256, 1024):
            if world == 1 and spp > 256:
                continue
            p = rtow.params(W, H, spp, seed=1, rank=0, world=world, max_depth=depth)
            ks = []
            for _ in range(2):
                st = ctx.render_tiles_device(cam, p, slab.data_ptr())
                ks.append(st.kernel_ms)
            pl = rtow.plan(p, ctx)
            k = min(ks)
            xs.append(spp)
            ys.append(k)
            print(f"world {world} depth {depth} spp {spp:5d}: kernel {k:8.3f} ms  rays {st.segments}  "
                  f"{st.segments / k / 1e3:8.1f} Mray/s  items of {pl.samples_per_chunk} n_big {pl.n_big} "
                  f"tail {pl.tail_samples}/{pl.n_tail}", flush=True)
        b, a = np.polyfit(xs[-3:], ys[-3:], 1)
        print(f"world {world} depth {depth}: last three points: {a:.2f} ms + {b:.4f} ms/spp", flush=True)
ctx.close()
