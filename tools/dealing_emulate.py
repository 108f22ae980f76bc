"""Price how work items are dealt to a wave's lanes (config 2's bench kernel)
on the oracle's own rays: does keeping a wave's lanes on neighbouring pixels
make its lockstep traversal cheaper?

Today every lane that needs work takes the next items of ONE global counter
(a wave's ballot + atomicAdd), so once the first items are done a wave's lanes
hold pixels spread over a band of the frame.  The alternatives keep a wave on
neighbouring items: the wave claims a range of items and its lanes refill from
that range (a wave-private queue), so its primary rays come from a few
adjacent pixels and its bounces start near each other.  All variants trace the
same rays' kind of work (random band of the frame, consecutive samples per
lane); tools/regroup_emu.c walks the uploaded SAH tree and the wave's cost is
the union of its lanes' slot paths per step (tools/regroup_emulate.py).

  wave<N>     one contiguous run of N-sample items (item = pixel * chunks +
              chunk, pixel-major in slab order) dealt wave by wave: a wave's
              64 lanes on ~9 adjacent pixels (N = 128) or on one pixel's 64
              chunks, refilling from the next pixels of its range (N = 16);
  shuffled<N> the SAME lanes (same items, same rays) shuffled across the
              waves, as the global counter mixes them -- so only the grouping
              differs between the two.

  python tools/dealing_emulate.py [iterations=200] [waves=48] [regions=4]
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import regroup_emulate as rg  # noqa: E402

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 200
WAVES = int(sys.argv[2]) if len(sys.argv) > 2 else 48
REGIONS = int(sys.argv[3]) if len(sys.argv) > 3 else 4


def main():
    lib = rg.build_emu()
    scene = rg.rtow.Scene.build("random_ned", n=487, image="synthetic", scene_seed=1)
    nodes, root, tshift, _ = rg.layout(scene)
    n_nodes = len(nodes) // 64
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
    cache = {}

    def sample_rays(fbpix, s):
        k = (fbpix, s)
        if k not in cache:
            x, y = fbpix % W, fbpix // W
            assert olib.rtow_oracle_trace_rays(scene.view_ptr, ctypes.byref(ocam), ctypes.byref(op), x, y, s,
                                               buf.ctypes.data, 64, ctypes.byref(cnt)) == 0
            r = buf[:cnt.value].copy()
            r[:, 0:3] = r[:, 0:3] - shift
            cache[k] = r
        return cache[k]

    def item_rays(fbpix, s0, spc):
        return np.concatenate([sample_rays(fbpix, s) for s in range(s0, s0 + spc)])

    def trace(rays):
        n = len(rays)
        rays = np.ascontiguousarray(rays, np.float32)
        codes = np.zeros((n, rg.MAXS), np.uint8)
        steps = np.zeros(n, np.int32)
        prim = np.zeros(n, np.uint32)
        bt = np.zeros(n, np.float32)
        assert lib.trace_rays(nodes.ctypes.data, n_nodes, root, tshift.ctypes.data, rays.ctypes.data, n,
                              codes.ctypes.data, rg.MAXS, steps.ctypes.data, prim.ctypes.data, bt.ctypes.data) == 0
        return codes, np.minimum(steps, rg.MAXS)

    def wave_cost(codes, steps):
        ms = int(steps.max())
        act = np.arange(ms)[None, :] < steps[:, None]
        c = codes[:, :ms]
        sph_b, sph_a = (((c & 1) != 0) & act).any(0), (((c & 2) != 0) & act).any(0)
        box_b, box_a = (((c & 1) == 0) & act).any(0), (((c & 2) == 0) & act).any(0)
        root_b, root_a = (((c & 4) != 0) & act).any(0), (((c & 8) != 0) & act).any(0)
        return (ms * rg.C_STEP + rg.C_BOX * (box_b.sum() + box_a.sum()) + rg.C_SPH * (sph_b.sum() + sph_a.sum()) +
                rg.C_ROOT * (root_b.sum() + root_a.sum())), int(act.sum()), ms

    rng = np.random.default_rng(13)
    # One contiguous run of items of the frame, dealt to WAVES waves in two
    # ways -- the SAME lanes (same items, same rays) either grouped wave by wave
    # in item order (a wave-private range) or shuffled across the waves (the
    # global counter's mixing) -- so only the grouping differs.
    tot = {k: np.zeros(4) for k in ("shuffled128", "wave128", "shuffled16", "wave16")}
    for region in range(REGIONS):
        b0 = int(rng.integers(0, W * H - WAVES * 64))
        lanes128 = [item_rays(int(idx_of[(b0 * 7 + j) // 7]), ((b0 * 7 + j) % 7) * 128, ITERS)[:ITERS]
                    for j in range(WAVES * 64)]

        def lanes16():
            """each wave a private queue of 16-sample items (pixel-major), lanes refilling in lane order"""
            out = []
            for w in range(WAVES):
                queue = iter(range((b0 + 9 * w) * 64, (b0 + 9 * w + 64) * 64))

                def nxt():
                    it = next(queue)
                    return item_rays(int(idx_of[it // 64]), (it % 64) * 16, 16)

                cur = [nxt() for _ in range(64)]
                pos = [0] * 64
                rows = [[] for _ in range(64)]
                for _ in range(ITERS):
                    for j in range(64):
                        if pos[j] >= len(cur[j]):
                            cur[j], pos[j] = nxt(), 0
                        rows[j].append(cur[j][pos[j]])
                        pos[j] += 1
                out += [np.stack(r) for r in rows]
            return out

        groups = {"128": lanes128, "16": lanes16()}
        perm = rng.permutation(WAVES * 64)
        for size, lanes in groups.items():
            R = np.stack(lanes)  # [WAVES * 64, ITERS, 7]
            codes, steps = trace(R.reshape(-1, 7))
            codes = codes.reshape(WAVES * 64, ITERS, -1)
            steps = steps.reshape(WAVES * 64, ITERS)
            for key, order in ((f"wave{size}", np.arange(WAVES * 64)), (f"shuffled{size}", perm)):
                for w in range(WAVES):
                    sel = order[64 * w:64 * w + 64]
                    for it in range(ITERS):
                        c, ls, ms = wave_cost(codes[sel, it], steps[sel, it])
                        tot[key] += [c, ls, ms, 64]
            print(f"region {region + 1}: items of {size} done", file=sys.stderr, flush=True)
    print(f"config 2: {REGIONS} regions x {WAVES} waves x {ITERS} iterations, per region one contiguous run of "
          f"items from a random place of the frame; VALU wave-instr per ray of the traversal (tools/regroup_emulate.py's costs)")
    for key, t in tot.items():
        base = tot["shuffled" + key.lstrip("shufledwav")][0] / tot["shuffled" + key.lstrip("shufledwav")][3]
        print(f"  {key:11s} traversal/ray {t[0] / t[3]:6.2f} ({t[0] / t[3] / base - 1:+.1%} vs shuffled)  "
              f"node steps/ray {t[1] / t[3]:5.2f}  lane efficiency {t[1] / (64 * t[2]):.3f}")


if __name__ == "__main__":
    main()
