"""Frames of one build with the SAH trees and with the reference trees: the
pixels that differ, and for the first few the first segment where the two
paths part (rtow_debug_trace_sample), next to the oracle's.
  python tools/tree_diff.py [scene] [W H SPP]   (default final_ned 1024 1024 16)"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402
from trace_diff import fmt  # noqa: E402


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "final_ned"
    W, H, spp = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1024, 1024, 16)
    sc = rtow.Scene.build(scene, image="synthetic")
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=1)
    ctxs, lins = [], []
    for tree in ("sah", "reference"):
        c = rtow.Context(0)
        c.set_tree(tree)
        c.upload(sc)
        ctxs.append(c)
        lins.append(c.render(cam, p)[1].reshape(-1, 3))
    d = np.abs(lins[0] - lins[1]).max(axis=1)
    bad = np.nonzero(d)[0]
    print(f"{len(bad)} pixels differ (max {d.max():.3g})")
    ocam = sio.RtowCamera.from_buffer_copy(bytes(cam))
    op = sio.RtowParams.from_buffer_copy(bytes(p))
    for fb in bad[:4]:
        x, y = int(fb % W), int(fb // W)
        for s in range(spp):
            g0 = ctxs[0].trace_sample(cam, p, x, y, s)
            g1 = ctxs[1].trace_sample(cam, p, x, y, s)
            n = min(len(g0), len(g1))
            k = next((i for i in range(n) if not np.array_equal(g0[i, :11], g1[i, :11])), None)
            if k is None and len(g0) == len(g1):
                continue
            k = n if k is None else k
            o = sio.oracle_trace(sc.view_ptr, ocam, op, x, y, s)
            print(f"pixel ({x},{y}) sample {s}: first difference at segment {k}")
            for i in range(max(0, k - 1), k + 1):
                for name, tr in (("sah", g0), ("ref", g1), ("oracle", o)):
                    if i < len(tr):
                        print(f"  {name:6s} [{i}] {fmt(tr[i])}")
            break


if __name__ == "__main__":
    main()
