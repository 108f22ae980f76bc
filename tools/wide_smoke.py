"""The 4-wide tree (MODE 7, RTOW_WIDE / RTOW_SPEC) on small frames first:
every variant's frame against the binary-tree kernel's (MODE 0), printing as
it goes, then one 1920x1080 frame per variant with its kernel time.
  python tools/wide_smoke.py [variants, e.g. 3 4 4:1 4:24]   (WIDE[:SPEC])"""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "ray-tracing-one-weekend_amd"))
import rtow  # noqa: E402

torch.cuda.init()
variants = sys.argv[1:] or ["3", "4", "4:1", "4:24"]
scene = rtow.Scene.build("random_ned", n=487, image="synthetic", scene_seed=1)
ref = rtow.Context(0)
ref.upload(scene)
for v in variants:
    w, _, sp = v.partition(":")
    os.environ["RTOW_WIDE"] = w
    os.environ["RTOW_SPEC"] = sp or "0"
    ctx = rtow.Context(0)
    ctx.upload(scene)
    os.environ.pop("RTOW_WIDE")
    os.environ.pop("RTOW_SPEC")
    for W, H, spp in [(64, 36, 1), (64, 36, 16), (320, 180, 16), (1920, 1080, 64)]:
        cam, p = rtow.camera_main(W, H), rtow.params(W, H, spp, seed=1)
        t0 = time.time()
        _, a, sa = ctx.render(cam, p)
        _, b, sb = ref.render(cam, p)
        same = np.array_equal(a.view(np.uint32), b.view(np.uint32))
        print(f"wide {v} {W}x{H}x{spp}: identical={same} segments {sa.segments}/{sb.segments} kernel {sa.kernel_ms:.2f} "
              f"vs {sb.kernel_ms:.2f} ms ({sa.segments / sa.kernel_ms / 1e3:.0f} vs {sb.segments / sb.kernel_ms / 1e3:.0f} "
              f"Mray/s) wall {time.time() - t0:.2f} s", flush=True)
    ctx.close()
