"""Price seeding the bench kernel's primary-ray traversal with a predicted hit
(config 2), on the oracle's own rays, before building it.

A lane renders a work item's 128 samples of ONE pixel in turn, so its primary
rays are nearly the same ray: the sphere the previous sample's primary ray hit
is a prediction for the next.  Testing that sphere first (its DNode slot, the
same Sphere::hit arithmetic) and starting trace_simple with its hit as the
record is exact -- the record key orders every candidate the same way, so the
closest hit and the frame do not change -- and the traversal then culls with
the final bound from its first step.  This tool measures what that saves:
every lane's rays (tools/regroup_emulate.py's "steady" dealing: random pixels
of a band of the frame, consecutive samples), traced by tools/regroup_emu.c
with and without the seed, costed as 64-lane lockstep waves.

  python tools/hit_seed_emulate.py [iterations=200] [blocks=8]
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import regroup_emulate as rg  # noqa: E402

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 200
BLOCKS = int(sys.argv[2]) if len(sys.argv) > 2 else 8
NONE = 15 << 28


def main():
    lib = rg.build_emu()
    lib.trace_rays_seeded.restype = ctypes.c_int
    lib.trace_rays_seeded.argtypes = lib.trace_rays.argtypes + [ctypes.c_void_p, ctypes.c_void_p]
    lib.sphere_t.restype = ctypes.c_float
    lib.sphere_t.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    scene = rg.rtow.Scene.build("random_ned", n=487, image="synthetic", scene_seed=1)
    nodes, root, tshift, _ = rg.layout(scene)
    n_nodes = len(nodes) // 64
    nf = nodes.view(np.float32).reshape(n_nodes, 16)
    nu = nodes.view(np.uint32).reshape(n_nodes, 16)
    slot_of = {}
    for i in range(n_nodes):
        for off in (0, 8):
            ref = int(nu[i, off + 7])
            if (ref >> 28) == 1:
                slot_of[ref] = np.ascontiguousarray(nf[i, off:off + 7])
    v = scene.view
    rec = np.ctypeslib.as_array(ctypes.cast(v.hitables, ctypes.POINTER(ctypes.c_uint8)),
                                shape=(v.n_hitables * 64,)).reshape(v.n_hitables, 64)
    shift = rec[v.root, 16:].view(np.float32)[0:3].copy()
    W, H, SPP = rg.W, rg.H, rg.SPP
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
    idx_of = rg.rtow.rank_pixels(W, H, 0, 1)
    rng = np.random.default_rng(11)

    def lane_rays(fbpix, s0, need):
        x, y = fbpix % W, fbpix // W
        out, prim, s = [], [], s0
        while sum(len(r) for r in out) < need:
            assert olib.rtow_oracle_trace_rays(scene.view_ptr, ctypes.byref(ocam), ctypes.byref(op), x, y, s % SPP,
                                               buf.ctypes.data, 64, ctypes.byref(cnt)) == 0
            out.append(buf[:cnt.value].copy())
            f = np.zeros(cnt.value, bool)
            f[0] = True
            prim.append(f)
            s += 1
        r = np.concatenate(out)[:need]
        r[:, 0:3] = r[:, 0:3] - shift
        return r, np.concatenate(prim)[:need]

    def trace(rays, seed_t=None, seed_ref=None):
        n = len(rays)
        rays = np.ascontiguousarray(rays, np.float32)
        codes = np.zeros((n, rg.MAXS), np.uint8)
        steps = np.zeros(n, np.int32)
        prim = np.zeros(n, np.uint32)
        bt = np.zeros(n, np.float32)
        st = np.ascontiguousarray(seed_t if seed_t is not None else np.zeros(n), np.float32)
        sr = np.ascontiguousarray(seed_ref if seed_ref is not None else np.full(n, NONE), np.uint32)
        assert lib.trace_rays_seeded(nodes.ctypes.data, n_nodes, root, tshift.ctypes.data, rays.ctypes.data, n,
                                     codes.ctypes.data, rg.MAXS, steps.ctypes.data, prim.ctypes.data, bt.ctypes.data,
                                     st.ctypes.data, sr.ctypes.data) == 0
        return codes, np.minimum(steps, rg.MAXS), prim, bt

    def wave_cost(codes, steps):
        ms = int(steps.max())
        act = np.arange(ms)[None, :] < steps[:, None]
        c = codes[:, :ms]
        sph_b, sph_a = (((c & 1) != 0) & act).any(0), (((c & 2) != 0) & act).any(0)
        box_b, box_a = (((c & 1) == 0) & act).any(0), (((c & 2) == 0) & act).any(0)
        root_b, root_a = (((c & 4) != 0) & act).any(0), (((c & 8) != 0) & act).any(0)
        return ms * rg.C_STEP + rg.C_BOX * (box_b.sum() + box_a.sum()) + rg.C_SPH * (sph_b.sum() + sph_a.sum()) + \
            rg.C_ROOT * (root_b.sum() + root_a.sum())

    tot = np.zeros(4)
    stats = np.zeros(6)
    for blk in range(BLOCKS):
        b0 = int(rng.integers(0, W * H - rg.BAND))
        lanes = [(int(idx_of[b0 + rng.integers(0, rg.BAND)]), int(rng.integers(0, SPP - 40))) for _ in range(512)]
        got = [lane_rays(px, s0, ITERS) for px, s0 in lanes]
        R = np.stack([g[0] for g in got]).reshape(-1, 7)
        P = np.stack([g[1] for g in got]).reshape(-1)
        codes, steps, prim, bt = trace(R)
        # the seed: the sphere the lane's previous primary ray hit, tested exactly on this one
        seed_t = np.zeros(len(R), np.float32)
        seed_ref = np.full(len(R), NONE, np.uint32)
        pr = prim.reshape(512, ITERS)
        pp = P.reshape(512, ITERS)
        n_pred = n_hit = n_same = 0
        for ln in range(512):
            last = NONE
            for it in range(ITERS):
                if not pp[ln, it]:
                    continue
                k = ln * ITERS + it
                if last != NONE and last in slot_of:
                    n_pred += 1
                    t = lib.sphere_t(slot_of[last].ctypes.data, np.ascontiguousarray(R[k]).ctypes.data)
                    if t > 0:
                        n_hit += 1
                        seed_t[k], seed_ref[k] = t, last
                        n_same += int(pr[ln, it] == last)
                last = int(pr[ln, it])
        codes2, steps2, prim2, bt2 = trace(R, seed_t, seed_ref)
        assert (prim2 == prim).all() and (bt2 == bt).all(), "the seed changed a record"
        c1, s1 = codes.reshape(512, ITERS, -1), steps.reshape(512, ITERS)
        c2, s2 = codes2.reshape(512, ITERS, -1), steps2.reshape(512, ITERS)
        for it in range(ITERS):
            for w in range(8):
                sel = slice(64 * w, 64 * w + 64)
                tot[0] += wave_cost(c1[sel, it], s1[sel, it])
                tot[1] += wave_cost(c2[sel, it], s2[sel, it])
                # the seed's own sphere test: once per wave iteration if a lane seeds
                tot[2] += (rg.C_SPH + rg.C_ROOT) if (seed_ref.reshape(512, ITERS)[sel, it] != NONE).any() else 0.0
        stats += [P.sum(), n_pred, n_hit, n_same, steps[P].sum(), steps2[P].sum()]
        print(f"block {blk + 1}/{BLOCKS}", file=sys.stderr, flush=True)
    n = BLOCKS * 512 * ITERS
    base = tot[0] / n
    seeded = (tot[1] + tot[2]) / n
    print(f"config 2, {BLOCKS} blocks x 512 lanes x {ITERS} iterations ('steady' dealing), VALU wave-instr per ray "
          f"(tools/regroup_emulate.py's costs)")
    print(f"primary rays {int(stats[0])} ({stats[0] / n:.3f} of the rays); predicted {int(stats[1])}, the prediction "
          f"hit {int(stats[2])}, was the closest hit {int(stats[3])}")
    print(f"node steps per primary ray: {stats[4] / stats[0]:.2f} -> {stats[5] / stats[0]:.2f} seeded")
    print(f"traversal issue per ray: {base:.2f} -> {tot[1] / n:.2f} + seed tests {tot[2] / n:.2f} = {seeded:.2f} "
          f"({seeded / base - 1:+.1%}); of the whole kernel (+ {rg.C_SHADE * 8 / 512:.1f} shading per ray): "
          f"{(seeded + rg.C_SHADE * 8 / 512) / (base + rg.C_SHADE * 8 / 512) - 1:+.1%}")


if __name__ == "__main__":
    main()
