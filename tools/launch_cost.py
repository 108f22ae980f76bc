"""Fixed cost per frame launch on one GPU: kernel (HIP events) and host
(rtow_stats.total_ms) time of the bench frame at a few spp; the intercept of
time vs spp is the per-launch cost.  python tools/launch_cost.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-one-weekend_amd"))
import rtow  # noqa: E402

W, H = 1920, 1080
torch.cuda.init()
scene = rtow.Scene.build("random_ned", n=487, image="synthetic", scene_seed=1)
cam = rtow.camera_main(W, H)
ctx = rtow.Context(0)
ctx.upload(scene)
slab = torch.zeros(rtow.rank_tile_count(W, H, 0, 1) * 64 * 4, dtype=torch.uint8, device="cuda")
ctx.render_tiles_device(cam, rtow.params(W, H, 4, seed=1), slab.data_ptr())  # warm
spps = [int(v) for v in os.environ.get("LC_SPP", "8,16,32,64,128").split(",")]
km, tm = [], []
for spp in spps:
    ks, ts = [], []
    for _ in range(3):
        st = ctx.render_tiles_device(cam, rtow.params(W, H, spp, seed=1, max_depth=int(os.environ.get("LC_DEPTH", "50"))), slab.data_ptr())
        ks.append(st.kernel_ms)
        ts.append(st.total_ms)
    km.append(min(ks))
    tm.append(min(ts))
    print(f"spp {spp:4d}: kernel {km[-1]:8.2f} ms  call {tm[-1]:8.2f} ms", flush=True)
bk, ak = np.polyfit(spps, km, 1)
bt, at = np.polyfit(spps, tm, 1)
print(f"kernel: {ak:.2f} ms + {bk:.4f} ms/spp | call: {at:.2f} ms + {bt:.4f} ms/spp", flush=True)
ctx.close()
