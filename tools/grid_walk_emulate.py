"""CPU emulation of MODE 8's grid walk (grid_walk, rtow_device.hip) on the
oracle's own final_ned paths, to price changes to the walk's structure
before building them.

Rays: every segment of random pixels' samples (rtow_oracle_trace_sample:
origin = the previous hit, direction from the next hit and its t), in the
grid's frame (world - the root Translate).  Each ray's walk is emulated as the
kernel does it: rows along v in the ray's order, in a row the cells along u,
a cell a candidate when the ray passes at a height its Box spans, the walk
stopping beyond the culling bound of the record; a candidate's Box is
"scanned" (its slab entry beyond tmin shrinks the record).  The lane's op
sequence then feeds a 64-lane lockstep model of the wave:

  current   each round every live lane walks to its next candidate (the wave
            steps max over lanes), then the wave scans the candidates together;
  spec K    while the round's slowest lane is still walking, lanes that have
            found a candidate walk on and queue up to K candidates; the wave
            then runs scan passes 1..K (a queued candidate whose cell starts
            beyond the record after the earlier scans is dropped).

Reported per variant: wave walk steps and wave scans per ray, the walk's lane
efficiency (lane steps / 64 wave steps; the instrumented kernel measures 0.219
for the current walk, profiles/r04/prof_counters_final_ned_grid.txt) and a
cost in VALU wave-instructions per ray (C_STEP per wave walk step, C_SCAN per
wave scan).

  python tools/grid_walk_emulate.py [pixels=400]"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "ray-tracing-one-weekend_amd"), os.path.join(HERE, "..", "tests")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402

NPX = int(sys.argv[1]) if len(sys.argv) > 1 else 400
C_STEP, C_SCAN = 30.0, 110.0
REL = 2.0 ** -18

scene = rtow.Scene.build("final_ned", n=1, image="synthetic", scene_seed=1)
v = scene.view
rec = np.ctypeslib.as_array(ctypes.cast(v.hitables, ctypes.POINTER(ctypes.c_uint8)),
                            shape=(v.n_hitables * 64,)).reshape(v.n_hitables, 64)
kind = rec[:, :16].view(np.uint32)[:, 0]
F = rec[:, 16:].view(np.float32).astype(np.float64)
shift = F[v.root, 0:3].copy()  # root Translate
boxes = np.flatnonzero(kind == 10)
BL, BH = F[boxes, 0:3], F[boxes, 3:6]
U0, V0, WU, WV, NU, NV = -1000.0, -1000.0, 100.0, 100.0, 20, 20
D = 100.0 * 2.0 ** -10
cell_box = -np.ones((NV, NU), int)
for k in range(len(boxes)):
    i = int(round((BL[k, 0] - U0) / WU))
    j = int(round((BL[k, 1] - V0) / WV))
    cell_box[j, i] = k
HLO, HHI = BL[:, 2].min(), BH[:, 2].max()
chlo = np.array([[BL[cell_box[j, i], 2] for i in range(NU)] for j in range(NV)])
chhi = np.array([[BH[cell_box[j, i], 2] for i in range(NU)] for j in range(NV)])
rhlo, rhhi = chlo.min(axis=1), chhi.max(axis=1)


def band(lo, hi, o, iv):
    if not np.isfinite(iv):
        return (-np.inf, np.inf) if lo <= o <= hi else (np.inf, -np.inf)
    a, b = (lo - o) * iv, (hi - o) * iv
    n, f = min(a, b), max(a, b)
    return n - abs(n) * REL, f + abs(f) * REL


def box_t(k, o, inv, tmin, bt):
    """The Box's slab entry (its six-side scan's nearest hit, for culling)."""
    t0, t1 = (BL[k] - o) * inv, (BH[k] - o) * inv
    tn, tf = np.minimum(t0, t1).max(), np.maximum(t0, t1).min()
    if tn > tf:
        return None
    t = tn if tn > tmin else tf
    return t if tmin < t < bt else None


def walk(o, d, tmin=0.001):
    """The lane's ops: a list of (steps to the candidate, cell entry c0, box) and
    the trailing steps after the last candidate; plus the closest Box t."""
    with np.errstate(divide="ignore"):
        inv = 1.0 / d
    ou, ov, oh = o
    du, dv, dh = d
    iu, iv, ih = inv
    u0, u1 = band(U0 - D, U0 + NU * WU + D, ou, iu)
    v0, v1 = band(V0 - D, V0 + NV * WV + D, ov, iv)
    h0, h1 = band(HLO - D, HHI + D, oh, ih)
    te, tx = max(u0, v0, h0, tmin), min(u1, v1, h1)
    bt = np.inf
    if not te <= min(tx, bt):
        return [], 0, bt
    sv, su = (-1 if dv < 0 else 1), (-1 if du < 0 else 1)
    vflat, uflat = not np.isfinite(iv), not np.isfinite(iu)

    def row_of(t, back):
        vv = t * dv + ov
        e = 2 * D + (abs(ov) + abs(vv)) * REL
        return int(min(max(np.floor((vv + back * e - V0) / WV), 0), NV - 1))

    Eu = D + (abs(ou) + abs(tx * du)) * REL
    Ev = D + (abs(ov) + abs(tx * dv)) * REL
    Eh = (abs(oh) + abs(tx * dh)) * REL
    j = row_of(te, -sv)
    jl = row_of(tx, sv)
    nrows = (jl - j) * sv + 1
    ncells, i, jr, ra, rb = 0, 0, 0, 0.0, 0.0
    cands, steps = [], 0
    while True:
        steps += 1
        bound = bt * (1 + 2 ** -9)
        if ncells <= 0:
            if nrows <= 0:
                break
            vlo = j * WV + V0
            t0, t1 = band(vlo - Ev, vlo + WV + Ev, ov, iv) if not vflat else band(vlo - Ev, vlo + WV + Ev, ov, iv)
            jr = j
            j += sv
            nrows -= 1
            if t0 > bound and not vflat:
                break
            ra, rb = max(t0, te), min(t1, tx, bound)
            if not ra <= rb:
                continue
            ha, hb = ra * dh + oh, rb * dh + oh
            if max(ha, hb) + Eh < rhlo[jr] or min(ha, hb) - Eh > rhhi[jr]:
                continue
            ua, ub = ra * du + ou, rb * du + ou
            fa = np.floor((min(ua, ub) - Eu - U0) / WU)
            fb = np.floor((max(ua, ub) + Eu - U0) / WU)
            ia, ib = int(min(max(fa, 0), NU - 1)), int(min(max(fb, 0), NU - 1))
            i = ia if su > 0 else ib
            ncells = ib - ia + 1
        ic = i
        i += su
        ncells -= 1
        ulo = ic * WU + U0
        c0, c1 = band(ulo - Eu, ulo + WU + Eu, ou, iu)
        c0, c1 = max(c0, ra), min(c1, rb, bound)
        if not c0 <= c1:
            if c0 > bound and not uflat:
                ncells = 0
            continue
        ha, hb = c0 * dh + oh, c1 * dh + oh
        if max(ha, hb) + Eh < chlo[jr, ic] or min(ha, hb) - Eh > chhi[jr, ic]:
            continue
        k = cell_box[jr, ic]
        cands.append((steps, c0, k))
        steps = 0
        t = box_t(k, o, inv, tmin, bt)
        if t is not None:
            bt = t
    return cands, steps, bt


W = H = 4096
cam, p = rtow.camera_main(W, H), rtow.params(W, H, 8, seed=1)
ocam, op = sio.RtowCamera.from_buffer_copy(bytes(cam)), sio.RtowParams.from_buffer_copy(bytes(p))
org = np.array(cam.origin[:], np.float64)
rng = np.random.default_rng(5)
paths = []
for _ in range(NPX):
    recs = sio.oracle_trace(scene.view_ptr, ocam, op, int(rng.integers(W)), int(rng.integers(H)), int(rng.integers(8)))
    prev = org.copy()
    path = []
    for r in recs:
        pt = r[3:6].astype(np.float64)
        d = (pt - prev) / float(r[2]) if r[0] == 1.0 else pt
        o = prev - shift
        cands, tail, bt = walk(o, d)
        path.append((o, d, cands, tail))
        if r[0] == 1.0:
            prev = pt
    paths.append(path)
segs = [s for pth in paths for s in pth]
n = len(segs)
lane_steps = sum(sum(c[0] for c in s[2]) + s[3] for s in segs)
print(f"{n} segments of {NPX} paths: walk steps {lane_steps / n:.2f} per ray (kernel: 2.34), candidates "
      f"{sum(len(s[2]) for s in segs) / n:.3f} per ray (kernel: 1.145 Box scans); rays with a walk "
      f"{sum(1 for s in segs if s[2] or s[3]) / n:.3f}")
hist = np.bincount([len(s[2]) for s in segs])
print("candidates per ray histogram:", hist[:10].tolist())


def model(order, K):
    """Lockstep cost of the wave for variant K (1 = current) over segments in `order`."""
    wave_steps = wave_scans = lane_st = 0
    for w0 in range(0, len(order) - 63, 64):
        lanes = [segs[q] for q in order[w0:w0 + 64]]
        # per lane: remaining candidate list (steps, c0, box) and tail steps
        rem = [list(L[2]) for L in lanes]
        tail = [L[3] for L in lanes]
        live = [bool(r) or t > 0 for r, t in zip(rem, tail)]
        while any(live):
            # a round: steps until every live lane has its next candidate (or finished)
            need = [(r[0][0] if r else tail[q]) if live[q] else 0 for q, r in enumerate(rem)]
            rnd = max(need)
            wave_steps += rnd
            queued = []
            for q in range(64):
                if not live[q]:
                    queued.append([])
                    continue
                budget, got = rnd, []
                while rem[q] and rem[q][0][0] <= budget and len(got) < K:
                    budget -= rem[q][0][0]
                    lane_st += rem[q][0][0]
                    got.append(rem[q].pop(0))
                    if rem[q]:  # the next candidate's steps already partly walked
                        pass
                if not got:  # walked its tail to the end
                    lane_st += tail[q]
                    tail[q] = 0
                    live[q] = False
                elif len(got) < K and rem[q] and budget > 0:
                    # walks on toward the next candidate with the steps left
                    rem[q][0] = (rem[q][0][0] - budget, rem[q][0][1], rem[q][0][2])
                    lane_st += budget
                elif not rem[q] and budget > 0 and len(got) < K:
                    used = min(budget, tail[q])
                    tail[q] -= used
                    lane_st += used
                queued.append(got)
                if not rem[q] and tail[q] == 0 and got:
                    live[q] = False
            depth = max(len(g) for g in queued)
            wave_scans += depth
    waves = len(order) // 64
    rays = waves * 64
    return wave_steps / rays, wave_scans / rays, lane_st / max(1, 64 * wave_steps)


# lanes hold segments of different paths and depths: a random order of all segments
order = rng.permutation(n)
for K in (1, 2, 3):
    ws, sc, eff = model(order, K)
    print(f"K={K}: wave walk steps {ws * 64:.2f} per wave-ray-batch, wave scans {sc * 64:.2f}; lane efficiency "
          f"{eff:.3f}; cost {C_STEP * ws + C_SCAN * sc:.2f} VALU wave-instr per ray")

# what the steps after a lane's last candidate cost (a lane that could tell
# right after its scan that the walk is over would not take them)
saved = [s for s in segs]
segs = [(o, d, c, (0 if c else t)) for (o, d, c, t) in saved]
ws, sc, eff = model(order, 1)
print(f"K=1 without the steps after the last candidate: wave walk steps {ws * 64:.2f}, scans {sc * 64:.2f}; "
      f"cost {C_STEP * ws + C_SCAN * sc:.2f}")
ws, sc, eff = model(order, 2)
print(f"K=2 without them: wave walk steps {ws * 64:.2f}, scans {sc * 64:.2f}; cost {C_STEP * ws + C_SCAN * sc:.2f}")
segs = saved
tails = np.array([s[3] for s in segs if s[2]])
print(f"steps after the last candidate: mean {tails.mean():.2f} over rays with candidates; "
      f"first-candidate steps mean {np.mean([s[2][0][0] for s in segs if s[2]]):.2f}")


# --- the wave-wide walk: the wave enumerates its lanes' walks
# together.  Phase R: every (lane, row) pair the lanes' row ranges hold is
# dealt over the wave's 64 lanes (a wave prefix sum over the row counts, the
# owner's ray read back from LDS), each testing the row band and heights and
# yielding the row's cell range; phase C the same for every (lane, row, cell)
# triple, a candidate flagged back to its owner; phase S each owner scans its
# candidates in walk order, skipping those that start beyond its record.  No
# lane waits on another's walk, but no record culls the walk either (the scans
# come after it).  Costs per wave round: a row or cell test as the kernel's
# step (C_STEP), plus the dealing (prefix sum over the wave, owner search,
# owner's 16 ray words from LDS, candidate flag back): C_DEAL; per walk the
# lanes' ray words staged to LDS: C_STAGE.
def walk_all(o, d, tmin=0.001):
    """Rows and cells the walk tests with no culling, and the candidates in walk order."""
    with np.errstate(divide="ignore"):
        inv = 1.0 / d
    ou, ov, oh = o
    du, dv, dh = d
    iu, iv, ih = inv
    u0, u1 = band(U0 - D, U0 + NU * WU + D, ou, iu)
    v0, v1 = band(V0 - D, V0 + NV * WV + D, ov, iv)
    h0, h1 = band(HLO - D, HHI + D, oh, ih)
    te, tx = max(u0, v0, h0, tmin), min(u1, v1, h1)
    if not te <= tx:
        return 0, 0, []
    sv, su = (-1 if dv < 0 else 1), (-1 if du < 0 else 1)

    def row_of(t, back):
        vv = t * dv + ov
        e = 2 * D + (abs(ov) + abs(vv)) * REL
        return int(min(max(np.floor((vv + back * e - V0) / WV), 0), NV - 1))

    Eu = D + (abs(ou) + abs(tx * du)) * REL
    Ev = D + (abs(ov) + abs(tx * dv)) * REL
    Eh = (abs(oh) + abs(tx * dh)) * REL
    j, jl = row_of(te, -sv), row_of(tx, sv)
    rows = cells = 0
    cands = []
    for jr in range(j, jl + sv, sv):
        rows += 1
        vlo = jr * WV + V0
        t0, t1 = band(vlo - Ev, vlo + WV + Ev, ov, iv)
        ra, rb = max(t0, te), min(t1, tx)
        if not ra <= rb:
            continue
        ha, hb = ra * dh + oh, rb * dh + oh
        if max(ha, hb) + Eh < rhlo[jr] or min(ha, hb) - Eh > rhhi[jr]:
            continue
        ua, ub = ra * du + ou, rb * du + ou
        ia = int(min(max(np.floor((min(ua, ub) - Eu - U0) / WU), 0), NU - 1))
        ib = int(min(max(np.floor((max(ua, ub) + Eu - U0) / WU), 0), NU - 1))
        for ic in (range(ia, ib + 1) if su > 0 else range(ib, ia - 1, -1)):
            cells += 1
            ulo = ic * WU + U0
            c0, c1 = band(ulo - Eu, ulo + WU + Eu, ou, iu)
            c0, c1 = max(c0, ra), min(c1, rb)
            if not c0 <= c1:
                continue
            ha, hb = c0 * dh + oh, c1 * dh + oh
            if max(ha, hb) + Eh < chlo[jr, ic] or min(ha, hb) - Eh > chhi[jr, ic]:
                continue
            cands.append((c0, cell_box[jr, ic]))
    return rows, cells, cands


C_DEAL, C_STAGE, C_SKIP = 22.0, 10.0, 6.0
allw = []
for pth in paths:
    for (o, d, _, _) in pth:
        with np.errstate(divide="ignore"):
            inv = 1.0 / d
        rows, cells, cands = walk_all(o, d)
        allw.append((rows, cells, cands, inv, o))
wr = wc = ws = wk = 0
walks = 0
for w0 in range(0, n - 63, 64):
    lanes = [allw[q] for q in order[w0:w0 + 64]]
    tr, tc = sum(L[0] for L in lanes), sum(L[1] for L in lanes)
    if tr:
        walks += 1
    wr += -(-tr // 64)
    wc += -(-tc // 64)
    # phase S: per lane its candidates in walk order, culled by its own record
    acts = []
    for rows, cells, cands, inv, o in lanes:
        bt, a = np.inf, []
        for c0, k in cands:
            if c0 > bt * (1 + 2 ** -9):
                a.append(0)
                continue
            a.append(1)
            t = box_t(k, o, inv, 0.001, bt)
            if t is not None:
                bt = t
        acts.append(a)
    for it in range(max(len(a) for a in acts)):
        if any(len(a) > it and a[it] for a in acts):
            ws += 1
        else:
            wk += 1
rays = (n // 64) * 64
cost = ((C_STEP + C_DEAL) * (wr + wc) + C_SCAN * ws + C_SKIP * wk + C_STAGE * walks) / rays
print(f"wave-wide walk: row rounds {wr / rays * 64:.2f}, cell rounds {wc / rays * 64:.2f}, wave scans "
      f"{ws / rays * 64:.2f} (+{wk / rays * 64:.2f} skip passes) per 64 rays; rows {sum(a[0] for a in allw) / n:.2f} and "
      f"cells {sum(a[1] for a in allw) / n:.2f} per ray unculled, candidates {sum(len(a[2]) for a in allw) / n:.3f}; "
      f"cost {cost:.2f} VALU wave-instr per ray (K=1 above: current walk)")
free = (C_STEP * (wr + wc) + C_SCAN * ws + C_SKIP * wk) / rays
print(f"  the same with the dealing and staging free: {free:.2f}; the wave scans alone: {C_SCAN * ws / rays:.2f}")
