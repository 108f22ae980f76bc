"""Whole-frame parity of every config against the C oracle (which is pinned
bit-exact to the reference): each config at its full resolution (config 5 at
1024x1024) and a reduced spp, every pixel compared.  Prints one JSON line per
config (per-channel RMS of the linear frame, max |diff|, pixels off by more
than 1e-3, share of bit-identical channel values, segment counts).

  python tools/validate.py [--out FILE] [--scenes a,b]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
EARTH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "input_images", "1_earth_8k.jpg")  # the benched scenes' texture (scenes.h:140)
sys.path[:0] = [os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402

CASES = [("three_sphere", 0, 200, 100, 8), ("random_ned", 487, 1920, 1080, 16), ("cornell", 0, 800, 800, 64),
         ("cornell_smoke", 0, 800, 800, 64), ("final_ned", 0, 1024, 1024, 16)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--scenes", default=None, help="comma-separated subset of the configs")
    args = ap.parse_args()
    import torch

    torch.cuda.init()
    threads, _ = rtow.host_threads()  # the CPUs this process may use (affinity, cgroup quota)
    ctx = rtow.Context(0)
    lines = []
    cases = [c for c in CASES if args.scenes is None or c[0] in args.scenes.split(",")]
    for name, n, W, H, spp in cases:
        scene = rtow.Scene.build(name, n=max(n, 1), image="jpeg", image_path=EARTH, scene_seed=1)  # as bench.py
        ctx.upload(scene)
        cam = rtow.camera_main(W, H)
        p = rtow.params(W, H, spp, seed=7)
        _, lin, st = ctx.render(cam, p)
        t0 = time.perf_counter()
        olin, _, oc = sio.oracle_render(scene.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                        sio.RtowParams.from_buffer_copy(bytes(p)), threads=threads)
        dt = time.perf_counter() - t0
        g = lin.reshape(-1, 3).astype(np.float64)
        o = olin.astype(np.float64)
        d = np.abs(g - o)
        out = {"scene": name, "width": W, "height": H, "spp": spp, "seed": 7,
               "rms_per_channel": [float(v) for v in np.sqrt(np.mean((g - o) ** 2, axis=0))],
               "max_abs_diff": float(d.max()), "pixels_off_1e-3": int((d.max(axis=1) > 1e-3).sum()),
               "pixels": W * H, "bit_identical_values": float(np.mean(g == o)),
               "segments_gpu": int(st.segments), "segments_oracle": int(oc.segments), "oracle_seconds": round(dt, 1)}
        print(json.dumps(out), flush=True)
        lines.append(out)
    ctx.close()
    if args.out:
        with open(args.out, "w") as f:
            f.write("".join(json.dumps(o) + "\n" for o in lines))


if __name__ == "__main__":
    main()
