"""How long a rank's share of config 2 drains at the end of its launch, by
plan: a discrete-event model of the persistent grid's work queue on the
oracle's own per-sample path lengths (tools/regroup_emulate.py's oracle).

Rank 0 of 8's pixels (a random subset of them, in the share's item order):
each pixel's samples' segment counts (rtow_oracle_trace_rays), so pixels
keep their own cost (sky 1 segment, glass up to 51).  LANES lanes (the grid
scaled down with the pixels) each take the next item of the plan when free;
an item costs the sum of its samples' segments, drawn from its pixel.  The
launch's makespan over (total work / LANES) is what the drain adds --
measured on the GPU as the intercept of kernel time vs spp
(profiles/r06/launch_cost_ranks.txt).  Per-item costs (refill, flush) are
not modelled.

  python tools/drain_emulate.py [pixels=2592] [samples per pixel=128]"""
import ctypes
import heapq
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import regroup_emulate as rg  # noqa: E402

NP = int(sys.argv[1]) if len(sys.argv) > 1 else 2592
NSP = int(sys.argv[2]) if len(sys.argv) > 2 else 128
LANES = NP * 262144 // 259200  # the grid's lanes per pixel of an 8-rank share
SPP = 1024


def pixel_costs():
    scene = rg.rtow.Scene.build("random_ned", n=487, image="synthetic", scene_seed=1)
    W, H = 1920, 1080
    cam, p = rg.rtow.camera_main(W, H), rg.rtow.params(W, H, SPP, seed=1)
    ocam, op = rg.sio.RtowCamera.from_buffer_copy(bytes(cam)), rg.sio.RtowParams.from_buffer_copy(bytes(p))
    olib = rg.sio.oracle()
    olib.rtow_oracle_trace_rays.restype = ctypes.c_int
    olib.rtow_oracle_trace_rays.argtypes = [ctypes.c_void_p, ctypes.POINTER(rg.sio.RtowCamera),
                                            ctypes.POINTER(rg.sio.RtowParams), ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.POINTER(ctypes.c_uint32)]
    buf = np.zeros((64, 7), np.float32)
    cnt = ctypes.c_uint32()
    idx = rg.rtow.rank_pixels(W, H, 0, 8)
    sel = np.sort(np.random.default_rng(3).choice(len(idx), NP, replace=False))
    out = np.zeros((NP, NSP))
    for i, k in enumerate(sel):
        fb = int(idx[k])
        for s in range(NSP):
            assert olib.rtow_oracle_trace_rays(scene.view_ptr, ctypes.byref(ocam), ctypes.byref(op), fb % W, fb // W, s,
                                               buf.ctypes.data, 64, ctypes.byref(cnt)) == 0
            out[i, s] = cnt.value
    return out


def plan(spc, tailk=1, order=None):
    """The items (pixel, samples) of the automatic plan with spc-sample items:
    full chunks pixel-major, then the halving tail of tailk..tailk+1 items'
    samples chunk-major (tailk 1 is rtow_device.hip's planParams)."""
    n_big = (SPP - tailk * spc) // spc
    R = SPP - n_big * spc
    sizes, k = [], 0
    while True:
        lk, lk1 = -(-R // (1 << k)), -(-R // (2 << k))
        if lk <= 1:
            sizes.append(lk)
            break
        sizes.append(lk - lk1)
        k += 1
    items = [(q, spc) for q in range(NP) for _ in range(n_big)]
    items += [(q, n) for n in sizes for q in (order if order is not None else range(NP))]
    return items, n_big, sizes


def makespan(pix, items, rng):
    costs = [pix[q, rng.integers(0, NSP, n)].sum() for q, n in items]
    heap = [0.0] * LANES
    end = 0.0
    for c in costs:
        t = heapq.heappop(heap) + c
        end = max(end, t)
        heapq.heappush(heap, t)
    return end / (sum(costs) / LANES)


def main():
    pix = pixel_costs()
    rng = np.random.default_rng(7)
    print(f"config 2, rank 0 of 8: {NP} pixels x {NSP} samples: {pix.mean():.3f} segments per sample, per pixel "
          f"{pix.mean(1).min():.2f} .. {pix.mean(1).max():.2f} (cv {pix.mean(1).std() / pix.mean():.2f}); {LANES} lanes")
    for name, kw in [("32-sample items, one-item tail (shipped)", dict(spc=32)), ("16, one-item tail", dict(spc=16)),
                     ("64, one-item tail", dict(spc=64)), ("32, two-item tail", dict(spc=32, tailk=2)),
                     ("128, one-item tail", dict(spc=128)),
                     ("32, the tail's costliest pixels first", dict(spc=32, order=np.argsort(-pix.mean(1))))]:
        items, nb, sizes = plan(**kw)
        r = [makespan(pix, items, rng) for _ in range(3)]
        print(f"  {name:40s} n_big {nb:3d} tail {sizes}: makespan / ideal {np.mean(r):.4f} ({min(r):.4f}-{max(r):.4f})",
              flush=True)


if __name__ == "__main__":
    main()
