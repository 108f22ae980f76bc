"""Price inter-wave ray regrouping for config 2's bench kernel before building it
(VERDICT r5 next #2).

The bench kernel (trace_kernel MODE 0, rtow_device.hip) runs 512-thread
blocks, 8 waves of 64 lanes; one lane owns one path and traces one segment per
iteration (trace_simple), so a wave's traversal costs the UNION of the code
paths its 64 lanes take, step by step, for as many steps as its longest ray.
Permuting rays inside a wave cannot change that (round 5, RTOW_REORDER);
moving them BETWEEN the block's waves can.  This tool models both on the
oracle's own config-2 rays:

  rays     every segment (origin, direction, time) of the samples the lanes
           own, from the C oracle (rtow_oracle_trace_rays: the reference's
           color() recursion, world frame), one lane's samples in sample order;
  tree     the SAH DNode tree the upload builds (RTOW_LAYOUT_DUMP), walked by
           tools/regroup_emu.c, a restatement of trace_simple (same slabs,
           culling bound, record key): per ray its node steps, and per step
           which of the four slot paths (slot b sphere / box, slot a sphere /
           box) it runs and whether its sphere roots are computed (disc > 0);
  dealing  lanes hold 128-sample work items (pixel, chunk).  "fresh": wave w
           takes items 64w .. 64w+63 (item = pixel * 7 + chunk, slab order),
           as at the start of a launch; "steady": every lane a random pixel of
           a band of 20000 consecutive slab pixels, as the persistent refill
           leaves them after the first items (a lane's items come from the
           global counter whenever it finishes one);
  waves    per iteration (a bounce of every lane): (a) today -- each wave
           traverses its own 64 lanes' segments; (b) regrouped -- the block's
           512 segments are sorted by a key (direction octant, then the Morton
           code of the origin) and dealt to the waves 64 at a time, each wave
           traversing for the owners (rays and records moved through LDS).

Cost of a wave's traversal = sum over its wave steps of C_STEP + C_BOX per box
slot path taken by any active lane + C_SPH per sphere slot path + C_ROOT per
sphere path whose roots any lane computes (VALU wave-instructions; the
per-path counts of the trace_simple loop in the shipped ISA, DESIGN.md
"Next, in order": ~19 per box slot, ~45 per sphere slot with a root).
Reported per ray: modelled traversal issue, lane efficiency per wave step,
sphere-paths per wave step (the instrumented kernel measures 16.0 node steps
per ray at 0.52 lane efficiency and 1.28 sphere paths per wave step,
DESIGN.md), and for (b) the barrier-bound time (the block waits for its
slowest wave every bounce: 8 x max over waves) plus the sort's modelled cost.

  gcc -O2 -shared -fPIC -ffp-contract=off -o tools/_build/regroup_emu.so tools/regroup_emu.c -lm
  python tools/regroup_emulate.py [iterations=160] [blocks=6]
"""
import ctypes
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "ray-tracing-one-weekend_amd"), os.path.join(REPO, "tests")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 160
BLOCKS = int(sys.argv[2]) if len(sys.argv) > 2 else 6
C_STEP, C_BOX, C_SPH, C_ROOT = 14.0, 19.0, 22.0, 23.0
C_SHADE = 1700.0  # per wave iteration outside the traversal (shading, refill, sums): ~0.32 of the cycles
C_SORT = 260.0    # per wave per bounce for (b): key, LDS counting sort over 512 keys, ray + record moves
W, H, SPP, NBIG, SPC = 1920, 1080, 1024, 7, 128
BAND = 20000
MAXS = 96


def build_emu():
    so = os.path.join(HERE, "_build", "regroup_emu.so")
    src = os.path.join(HERE, "regroup_emu.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(so), exist_ok=True)
        subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-ffp-contract=off", "-o", so, src, "-lm"], check=True)
    lib = ctypes.CDLL(so)
    lib.trace_rays.restype = ctypes.c_int
    lib.trace_rays.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p]
    return lib


def layout(scene):
    """The uploaded arrays of a simple scene: DNodes, tshift, bvh_root."""
    path = os.path.join(tempfile.mkdtemp(), "layout.bin")
    os.environ["RTOW_LAYOUT_DUMP"] = path
    try:
        sio.scene_check(scene)
    finally:
        os.environ.pop("RTOW_LAYOUT_DUMP")
    b = open(path, "rb").read()
    parts, off = [], 0
    while off < len(b):
        n = int(np.frombuffer(b, np.uint64, 1, off)[0])
        parts.append(b[off + 8:off + 8 + n])
        off += 8 + n
    nodes = np.frombuffer(parts[1], np.uint8).copy()
    scal = np.frombuffer(parts[31], np.uint32)
    tshift = np.frombuffer(parts[32], np.float32).copy()
    return nodes, int(scal[14]), tshift, int(scal[7])


def main():
    lib = build_emu()
    scene = rtow.Scene.build("random_ned", n=487, image="synthetic", scene_seed=1)
    nodes, root, tshift, simple = layout(scene)
    assert simple == 1
    n_nodes = len(nodes) // 64
    v = scene.view
    rec = np.ctypeslib.as_array(ctypes.cast(v.hitables, ctypes.POINTER(ctypes.c_uint8)),
                                shape=(v.n_hitables * 64,)).reshape(v.n_hitables, 64)
    shift = rec[v.root, 16:].view(np.float32)[0:3].copy()  # the root Translate (main.cpp:132)
    cam, p = rtow.camera_main(W, H), rtow.params(W, H, SPP, seed=1)
    ocam, op = sio.RtowCamera.from_buffer_copy(bytes(cam)), sio.RtowParams.from_buffer_copy(bytes(p))
    olib = sio.oracle()
    olib.rtow_oracle_trace_rays.restype = ctypes.c_int
    olib.rtow_oracle_trace_rays.argtypes = [ctypes.c_void_p, ctypes.POINTER(sio.RtowCamera),
                                            ctypes.POINTER(sio.RtowParams), ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.POINTER(ctypes.c_uint32)]
    buf = np.zeros((64, 7), np.float32)
    cnt = ctypes.c_uint32()
    idx_of = rtow.rank_pixels(W, H, 0, 1)  # slab position -> framebuffer index

    def lane_rays(fbpix, s0, need):
        """segments of samples s0, s0+1, ... of one pixel until `need` rays"""
        x, y = fbpix % W, fbpix // W
        out, s = [], s0
        while sum(len(r) for r in out) < need:
            rc = olib.rtow_oracle_trace_rays(scene.view_ptr, ctypes.byref(ocam), ctypes.byref(op), x, y, s % SPP,
                                             buf.ctypes.data, 64, ctypes.byref(cnt))
            assert rc == 0
            out.append(buf[:cnt.value].copy())
            s += 1
        r = np.concatenate(out)[:need]
        r[:, 0:3] = r[:, 0:3] - shift  # into the BVH frame (root_ray: o - offset)
        return r

    def trace(rays):
        n = len(rays)
        rays = np.ascontiguousarray(rays, np.float32)
        codes = np.zeros((n, MAXS), np.uint8)
        steps = np.zeros(n, np.int32)
        prim = np.zeros(n, np.uint32)
        bt = np.zeros(n, np.float32)
        rc = lib.trace_rays(nodes.ctypes.data, ctypes.c_uint32(n_nodes), ctypes.c_uint32(root),
                            tshift.ctypes.data, rays.ctypes.data, ctypes.c_int(n), codes.ctypes.data,
                            ctypes.c_int(MAXS), steps.ctypes.data, prim.ctypes.data, bt.ctypes.data)
        assert rc == 0, rc
        return codes, np.minimum(steps, MAXS), steps

    def wave_cost(codes, steps):
        """lockstep traversal cost of one wave's rays"""
        ms = int(steps.max()) if len(steps) else 0
        act = np.arange(ms)[None, :] < steps[:, None]
        c = codes[:, :ms]
        any_ = lambda bit: ((c & bit) != 0) & act  # noqa: E731
        sph_b, sph_a = any_(1).any(0), any_(2).any(0)
        box_b, box_a = (((c & 1) == 0) & act).any(0), (((c & 2) == 0) & act).any(0)
        root_b, root_a = any_(4).any(0), any_(8).any(0)
        cost = ms * C_STEP + C_BOX * (box_b.sum() + box_a.sum()) + C_SPH * (sph_b.sum() + sph_a.sum()) + \
            C_ROOT * (root_b.sum() + root_a.sum())
        return cost, ms, int(act.sum()), int(sph_b.sum() + sph_a.sum())

    def morton(o, lo, hi, bits=7):
        q = np.clip(((o - lo) / (hi - lo) * (1 << bits)).astype(np.int64), 0, (1 << bits) - 1)
        code = np.zeros(len(o), np.int64)
        for b in range(bits):
            for ax in range(3):
                code |= ((q[:, ax] >> b) & 1) << (3 * b + ax)
        return code

    rng = np.random.default_rng(7)
    results = {}
    for dealing in ("fresh", "steady"):
        tot = {k: np.zeros(6) for k in ("a", "b_oct_morton", "b_morton", "b_steps_oracle")}
        n_rays = 0
        for blk in range(BLOCKS):
            # the block's 512 lanes: (framebuffer pixel, first sample)
            if dealing == "fresh":
                base = int(rng.integers(0, (W * H * NBIG) // 2)) // 512 * 512
                items = base + np.arange(512)
                lanes = [(int(idx_of[it // NBIG]), int((it % NBIG) * SPC + rng.integers(0, SPC - 40)))
                         for it in items]
            else:
                b0 = int(rng.integers(0, W * H - BAND))
                lanes = [(int(idx_of[b0 + rng.integers(0, BAND)]), int(rng.integers(0, SPP - 40))) for _ in range(512)]
            R = np.stack([lane_rays(px, s0, ITERS) for px, s0 in lanes])  # [512, ITERS, 7]
            codes, steps, raw = trace(R.reshape(-1, 7))
            codes = codes.reshape(512, ITERS, MAXS)
            steps = steps.reshape(512, ITERS)
            n_rays += 512 * ITERS
            lo, hi = R[:, :, 0:3].reshape(-1, 3).min(0), R[:, :, 0:3].reshape(-1, 3).max(0)
            for it in range(ITERS):
                c_it, s_it, r_it = codes[:, it], steps[:, it], R[:, it]
                # (a) today: wave w = lanes 64w .. 64w+63
                for key, order in (("a", np.arange(512)),
                                   ("b_oct_morton", None), ("b_morton", None), ("b_steps_oracle", None)):
                    if key == "b_oct_morton":
                        d = r_it[:, 3:6]
                        octant = (d[:, 0] < 0) * 1 + (d[:, 1] < 0) * 2 + (d[:, 2] < 0) * 4
                        order = np.lexsort((morton(r_it[:, 0:3], lo, hi), octant))
                    elif key == "b_morton":
                        order = np.argsort(morton(r_it[:, 0:3], lo, hi), kind="stable")
                    elif key == "b_steps_oracle":  # (an upper bound: rays sorted by their own step count)
                        order = np.argsort(s_it, kind="stable")
                    costs = []
                    for w in range(8):
                        sel = order[64 * w:64 * w + 64]
                        cst, ms, lane_steps, sph_paths = wave_cost(c_it[sel], s_it[sel])
                        costs.append(cst)
                        tot[key][1] += ms
                        tot[key][2] += lane_steps
                        tot[key][3] += sph_paths
                    tot[key][0] += sum(costs)
                    tot[key][4] += 8 * max(costs)
            print(f"[{dealing}] block {blk + 1}/{BLOCKS} done", file=sys.stderr, flush=True)
        results[dealing] = (tot, n_rays)
    print(f"config 2 (random_ned n=487, SAH DNodes {n_nodes}), {BLOCKS} blocks x 512 lanes x {ITERS} iterations per "
          f"dealing; costs in VALU wave-instructions per ray (C_STEP {C_STEP}, C_BOX {C_BOX}, C_SPH {C_SPH}, "
          f"C_ROOT {C_ROOT}; shading {C_SHADE} and sort {C_SORT} per wave iteration)")
    for dealing, (tot, n_rays) in results.items():
        a = tot["a"]
        base_total = (a[0] + C_SHADE * 8 * n_rays / 512) / n_rays
        print(f"\n{dealing}: {n_rays} rays")
        print(f"  {'variant':16s} {'trav/ray':>9s} {'steps/ray':>9s} {'lane eff':>8s} {'sph paths/step':>14s} "
              f"{'issue/ray':>9s} {'vs a':>7s} {'(no sort)':>9s} {'barrier/ray':>11s} {'vs a':>7s}")
        for key, t in tot.items():
            trav = t[0] / n_rays
            steps_ray = t[2] / n_rays
            eff = t[2] / (64 * t[1])
            sph = t[3] / t[1]
            extra = 0.0 if key == "a" else C_SORT * 8 * n_rays / 512 / n_rays
            issue = trav + C_SHADE * 8 / 512 + extra
            barrier = t[4] / n_rays + C_SHADE * 8 / 512 + extra
            a_barrier = a[0] / n_rays + C_SHADE * 8 / 512
            print(f"  {key:16s} {trav:9.2f} {steps_ray:9.2f} {eff:8.3f} {sph:14.2f} {issue:9.2f} "
                  f"{issue / base_total - 1:+7.1%} {(issue - extra) / base_total - 1:+9.1%} {barrier:11.2f} "
                  f"{barrier / a_barrier - 1:+7.1%}")


if __name__ == "__main__":
    main()
