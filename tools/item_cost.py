"""Where a general scene's time goes: the frame with one top-level list item
removed at a time (segments change too, so both are printed).
  python tools/item_cost.py [scene] [W H SPP]   (default final_ned 512 512 8)"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")]

import rtow  # noqa: E402
import scene_io as sio  # noqa: E402


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "final_ned"
    W, H, spp = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (512, 512, 8)
    d = sio.scene_dict(rtow.Scene.build(scene, image="synthetic"))
    h = d["hitables"]
    lst = int(h[d["root"]]["a"]) if h[d["root"]]["kind"] == sio.HIT_TRANSLATE else int(d["root"])
    first, count = int(h[lst]["a"]), int(h[lst]["b"])
    items = [int(r) for r in d["refs"][first:first + count]]
    ctx = rtow.Context(0)
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=1)
    for drop in [None] + list(range(count)):
        keep = [it for k, it in enumerate(items) if k != drop]
        e = sio.with_items(d, lst, keep)
        sc = sio.ArrayScene(e)
        try:
            ctx.upload(sc)
        except rtow.RtowError as err:
            print(f"drop {drop}: {err}")
            continue
        ctx.render(cam, p, linear=False)
        ms = min(ctx.render(cam, p, linear=False)[2].kernel_ms for _ in range(2))
        st = ctx.render(cam, p, linear=False)[2]
        name = "none" if drop is None else f"{drop} (kind {int(h[items[drop]]['kind'])})"
        print(f"drop {name:14s}: {ms:7.2f} ms  {st.segments / 1e6:7.2f} M segments  "
              f"{st.segments / ms / 1e3:6.0f} Mray/s  {ms / st.segments * 1e9:6.2f} ns/segment", flush=True)


if __name__ == "__main__":
    main()
