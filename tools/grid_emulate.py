"""CPU emulation of a uniform-grid traversal for the random scene (config 2),
on the oracle's own paths -- the question: would a 2D grid over the small
spheres (the big ones tested by every lane in place) issue fewer wave
instructions than the binary SAH tree's traversal?

Rays: every segment of random pixels' samples, from rtow_oracle_trace_sample
(origin = the previous hit, direction from the next hit and its t; the BVH's
frame = world - the root Translate).  Each ray's walk is emulated exactly
(closest hit checked against brute force); the wave cost comes from a
lockstep model: 64 lanes, each taking its paths' segments one per iteration,
a wave step costing C_D if any lane advances its cell walk and C_S if any lane
tests a sphere, plus the big spheres' in-place tests every iteration.

  python tools/grid_emulate.py [cell=1.0] [pixels=600] [big_radius=2]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "ray-tracing-one-weekend_amd"), os.path.join(HERE, "..", "tests")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402

CELL = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
NPX = int(sys.argv[2]) if len(sys.argv) > 2 else 600
BIG = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
C_S, C_D = 45.0, 25.0  # VALU wave-instructions: a sphere test with its root, a cell step

scene = rtow.Scene.build("random_ned", n=487, image="synthetic", scene_seed=1)
v = scene.view
import ctypes  # noqa: E402

hit = np.ctypeslib.as_array(ctypes.cast(v.hitables, ctypes.POINTER(ctypes.c_uint8)), shape=(v.n_hitables * 64,))
rec = hit.reshape(v.n_hitables, 64)
kind = rec[:, :16].view(np.uint32)[:, 0]
F = rec[:, 16:].view(np.float32).astype(np.float64)
sph = []  # c0, c1, r
for i in range(v.n_hitables):
    if kind[i] == 1:
        sph.append((F[i, 0:3], F[i, 0:3], F[i, 3]))
    elif kind[i] == 2:
        sph.append((F[i, 0:3], F[i, 3:6], F[i, 8]))
C0 = np.array([s[0] for s in sph])
C1 = np.array([s[1] for s in sph])
RAD = np.array([s[2] for s in sph])
big = np.flatnonzero(RAD >= BIG)
small = np.flatnonzero(RAD < BIG)
lo = np.minimum(C0[small], C1[small]) - RAD[small, None]
hi = np.maximum(C0[small], C1[small]) + RAD[small, None]
g0, g1 = lo.min(axis=0), hi.max(axis=0)
nu, nv = int(np.ceil((g1[0] - g0[0]) / CELL)), int(np.ceil((g1[1] - g0[1]) / CELL))
cells = [[[] for _ in range(nu)] for _ in range(nv)]
for k, s in enumerate(small):
    for j in range(int((lo[k, 1] - g0[1]) // CELL), int((hi[k, 1] - g0[1]) // CELL) + 1):
        for i in range(int((lo[k, 0] - g0[0]) // CELL), int((hi[k, 0] - g0[0]) // CELL) + 1):
            cells[min(j, nv - 1)][min(i, nu - 1)].append(s)
hz = np.full((nv, nu, 2), np.nan)
for j in range(nv):
    for i in range(nu):
        if cells[j][i]:
            ks = [np.searchsorted(small, s) for s in cells[j][i]]
            hz[j, i] = lo[ks, 2].min(), hi[ks, 2].max()
occ = [len(c) for row in cells for c in row]
print(f"grid {nu}x{nv} cells of {CELL}: {len(small)} small spheres, {len(big)} big (r >= {BIG}); "
      f"spheres per non-empty cell {np.mean([o for o in occ if o]):.2f}, max {max(occ)}, empty {occ.count(0)}")


def sph_t(j, o, d, time, tmin=0.001):
    c = C0[j] + time * (C1[j] - C0[j])
    oc = o - c
    a, b, cc = d @ d, d @ oc, oc @ oc - RAD[j] ** 2
    disc = b * b - a * cc
    if disc <= 0:
        return None
    sq = np.sqrt(disc)
    for t in ((-b - sq) / a, (-b + sq) / a):
        if tmin < t < 3.4e38:
            return t
    return None


def walk(o, d, time, tmin=0.001):
    """(closest t, sphere, ops): ops is the lane's op string, 'D' a cell step, 'S' a sphere test."""
    best, bj = np.inf, None
    for j in big:  # in place, every lane
        t = sph_t(j, o, d, time)
        if t is not None and t < best:
            best, bj = t, j
    ops = []
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t0s, t1s = (g0 - o) * inv, (g1 - o) * inv
    tn = np.where(np.isfinite(t0s), np.minimum(t0s, t1s), np.where((g0 <= o) & (o <= g1), -np.inf, np.inf))
    tf = np.where(np.isfinite(t0s), np.maximum(t0s, t1s), np.where((g0 <= o) & (o <= g1), np.inf, -np.inf))
    te, tx = max(tn.max(), tmin), tf.min()
    if not te <= min(tx, best):
        return best, bj, ops
    p = o + te * d
    i = min(max(int((p[0] - g0[0]) // CELL), 0), nu - 1)
    j = min(max(int((p[1] - g0[1]) // CELL), 0), nv - 1)
    si, sj = (1 if d[0] > 0 else -1), (1 if d[1] > 0 else -1)
    tcur = te
    while 0 <= i < nu and 0 <= j < nv and tcur <= min(tx, best * (1 + 2 ** -9)):
        ops.append("D")
        # the cell's exit
        bx = g0[0] + (i + (si > 0)) * CELL
        by = g0[1] + (j + (sj > 0)) * CELL
        with np.errstate(divide="ignore", invalid="ignore"):
            txx = (bx - o[0]) * inv[0] if np.isfinite(inv[0]) else np.inf
            tyy = (by - o[1]) * inv[1] if np.isfinite(inv[1]) else np.inf
        texit = min(txx, tyy, tx)
        if cells[j][i]:
            za, zb = o[2] + tcur * d[2], o[2] + texit * d[2]
            if max(za, zb) >= hz[j, i, 0] and min(za, zb) <= hz[j, i, 1]:
                for s in cells[j][i]:
                    ops.append("S")
                    t = sph_t(s, o, d, time)
                    if t is not None and t < best:
                        best, bj = t, s
        tcur = texit
        if txx < tyy:
            i += si
        else:
            j += sj
    return best, bj, ops


W, H = 1920, 1080
cam, p = rtow.camera_main(W, H), rtow.params(W, H, 4, seed=1)
ocam, op = sio.RtowCamera.from_buffer_copy(bytes(cam)), sio.RtowParams.from_buffer_copy(bytes(p))
org, shift = np.array(cam.origin[:], np.float64), np.array([0.0, 0.0, 1000.0])
rng = np.random.default_rng(3)
paths, bad, nseg = [], 0, 0
for _ in range(NPX):
    px, py, smp = int(rng.integers(W)), int(rng.integers(H)), int(rng.integers(4))
    recs = sio.oracle_trace(scene.view_ptr, ocam, op, px, py, smp)
    prev = org.copy()
    path = []
    for r in recs:
        pt = r[3:6].astype(np.float64)
        d = (pt - prev) / float(r[2]) if r[0] == 1.0 else pt
        time = float(rng.random())
        bt, bj, ops = walk(prev - shift, d, time)
        # brute force over every sphere
        tb, jb = np.inf, None
        for j in range(len(RAD)):
            t = sph_t(j, prev - shift, d, time)
            if t is not None and t < tb:
                tb, jb = t, j
        bad += (bj is None) != (jb is None) or (jb is not None and abs(bt - tb) > 1e-9 * max(1.0, tb))
        path.append(ops)
        nseg += 1
        if r[0] == 1.0:
            prev = pt
    paths.append(path)

ops_all = [o for pth in paths for o in pth]
print(f"{nseg} segments of {NPX} paths; closest-hit mismatches vs brute force {bad}")
print(f"per ray: cell steps {np.mean([o.count('D') for o in ops_all]):.2f}, sphere tests "
      f"{np.mean([o.count('S') for o in ops_all]):.2f} (+{len(big)} in place); max ops {max(len(o) for o in ops_all)}")

# lockstep wave model
cost, rays = 0.0, 0
queue = list(range(len(paths)))
rng.shuffle(queue)
lanes = [[] for _ in range(64)]
qi = 0
while True:
    segs = []
    for L in range(64):
        if not lanes[L] and qi < len(queue):
            lanes[L] = list(paths[queue[qi]])
            qi += 1
        if lanes[L]:
            segs.append(lanes[L].pop(0))
    if not segs:
        break
    rays += len(segs)
    cost += len(big) * C_S
    steps = max(len(s) for s in segs)
    for k in range(steps):
        kinds = {s[k] for s in segs if k < len(s)}
        cost += (C_D if "D" in kinds else 0) + (C_S if "S" in kinds else 0)
print(f"lockstep model: {cost / rays:.1f} VALU wave-instructions per ray in the traversal "
      f"(C_S {C_S}, C_D {C_D}); the SAH tree kernel measures ~55.7 (0.682 x 81.6, profiles/r04)")
