"""Which top-level item of a scene makes the GPU differ from the oracle?

Renders the scene with its root list cut down to subsets of items (root
Translate kept), GPU vs oracle, and prints the per-channel RMS of each.
  python tools/isolate.py [scene] [W H SPP]   (default final_ned 48 48 16)"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402

HIT_LIST = 9


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "final_ned"
    W, H, spp = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (48, 48, 16)
    d = sio.scene_dict(rtow.Scene.build(scene, image="synthetic"))
    h = d["hitables"]
    root = d["root"]
    lst = h[root]["a"] if h[root]["kind"] == sio.HIT_TRANSLATE else root
    assert h[lst]["kind"] == HIT_LIST
    first, count = int(h[lst]["a"]), int(h[lst]["b"])
    items = [int(r) for r in d["refs"][first:first + count]]
    ctx = rtow.Context(0)
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=5)
    subsets = [[k] for k in range(count)] + [list(range(count))]
    if len(sys.argv) > 5:
        subsets = [[int(x) for x in s.split(",")] for s in sys.argv[5:]]
    for sub in subsets:
        e = {k: (v.copy() if hasattr(v, "copy") else v) for k, v in d.items()}
        refs = np.concatenate([e["refs"], np.array([items[k] for k in sub], np.uint32)])
        e["refs"] = refs
        e["hitables"][lst]["a"] = len(d["refs"])
        e["hitables"][lst]["b"] = len(sub)
        sc = sio.ArrayScene(e)
        ctx.upload(sc)
        _, lin, st = ctx.render(cam, p)
        olin, _, oc = sio.oracle_render(sc.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                        sio.RtowParams.from_buffer_copy(bytes(p)))
        lin = lin.reshape(-1, 3).astype(np.float64)
        rms = np.sqrt(np.mean((lin - olin) ** 2, axis=0))
        bad = int((np.abs(lin - olin).max(axis=1) > 1e-3).sum())
        kinds = [int(h[items[k]]["kind"]) for k in sub]
        print(f"items {sub} kinds {kinds}: rms {rms} pixels>1e-3 {bad} segs gpu {st.segments} oracle {oc.segments}",
              flush=True)


if __name__ == "__main__":
    main()
