"""Per-sample path diff, GPU vs oracle (rtow_debug_trace_sample /
rtow_oracle_trace_sample): for the pixels where the frames differ, find the
samples whose paths differ and print the first diverging segment.

  python tools/trace_diff.py SCENE [W H SPP] [--ground]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402

FIELDS = "hit depth t p0 p1 p2 n0 n1 n2 mat ctr ok".split()


def fmt(r):
    return " ".join(f"{k}={v:.9g}" for k, v in zip(FIELDS[:11], r[:11]))


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    scene = args[0] if args else "final_ned"
    W, H, spp = (int(v) for v in args[1:4]) if len(args) >= 4 else (48, 48, 16)
    d = sio.scene_dict(rtow.Scene.build(scene, n=int(os.environ.get("TD_N", "100")), image="synthetic"))
    if "--ground" in sys.argv:  # final_ned's ground item only
        h = d["hitables"]
        lst = int(h[d["root"]]["a"])
        d = sio.with_items(d, lst, [int(d["refs"][int(h[lst]["a"])])])
    sc = sio.ArrayScene(d)
    ctx = rtow.Context(0)
    ctx.upload(sc)
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=int(os.environ.get("TD_SEED", "5")))
    ocam = sio.RtowCamera.from_buffer_copy(bytes(cam))
    op = sio.RtowParams.from_buffer_copy(bytes(p))
    _, lin, _ = ctx.render(cam, p)
    olin, _, _ = sio.oracle_render(sc.view_ptr, ocam, op, threads=16)
    diff = np.abs(lin.reshape(-1, 3).astype(np.float64) - olin).max(axis=1)
    bad = np.argsort(-diff)[: int(os.environ.get("TD_PIXELS", "4"))]
    shown = 0
    for fb in bad:
        if diff[fb] == 0:
            break
        x, y = int(fb % W), int(fb // W)
        for s in range(spp):
            g = ctx.trace_sample(cam, p, x, y, s)
            o = sio.oracle_trace(sc.view_ptr, ocam, op, x, y, s)
            n = min(len(g), len(o))
            k = next((i for i in range(n) if not np.array_equal(g[i, :11], o[i, :11])), None)
            if k is None and len(g) == len(o):
                continue
            k = n if k is None else k
            print(f"pixel ({x},{y}) sample {s}: {len(g)} gpu / {len(o)} oracle segments, first difference at {k}")
            for i in range(max(0, k - 1), min(k + 2, max(len(g), len(o)))):
                if i < len(g):
                    print(f"  gpu    [{i}] {fmt(g[i])}")
                if i < len(o):
                    print(f"  oracle [{i}] {fmt(o[i])}")
            shown += 1
            break
    print(f"{shown} diverging samples shown")


if __name__ == "__main__":
    main()
