"""CPU emulation of the 4-wide tree's traversal (trace_wide, MODE 7) on the
oracle's own paths: builds the tree through the library (RTOW_WIDE=k,
RTOW_WIDE_DUMP), rebuilds every segment of random pixels' first samples
from rtow_oracle_trace_sample (origin = the previous hit, direction from the
next hit and its t), walks the tree as the kernel does (nearest child next,
the others pushed far to near, leaves' spheres in a loop) and reports inner
steps, leaf steps and sphere tests per ray -- plus a check that the walk finds
the brute-force closest sphere on every segment.
  python tools/wide_emulate.py [k=4] [pixels=150]"""
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "ray-tracing-one-weekend_amd"), os.path.join(HERE, "..", "tests")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402

k = sys.argv[1] if len(sys.argv) > 1 else "4"
npx = int(sys.argv[2]) if len(sys.argv) > 2 else 150
dump = os.path.join(tempfile.mkdtemp(), "wide.bin")
subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r); import rtow; "
                "rtow.Scene.build('random_ned', n=487, image='synthetic', scene_seed=1).check()"
                % os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")],
               env=dict(os.environ, RTOW_WIDE=k, RTOW_LAYOUT_INFO="1", RTOW_WIDE_DUMP=dump), check=True,
               capture_output=True)
buf = open(dump, "rb").read()
n, root, need, nsph = struct.unpack_from("4I", buf, 0)
tshift = np.frombuffer(buf, np.float32, 3, 16).astype(np.float64)
off = 28
Wb = np.frombuffer(buf, np.uint8, n * 128, off).reshape(n, 128)
F = Wb.view(np.float32)[:, :28].astype(np.float64)
R = Wb.view(np.uint32)[:, 28:32]
off += n * 128
SF = np.frombuffer(buf, np.uint8, nsph * 48, off).reshape(nsph, 48).view(np.float32).astype(np.float64)
NONE, LEAF = 0xFFFF, 0x8000


def slab(lo, hi, o, inv, tmin, btc):
    t0, t1 = (lo - o) * inv, (hi - o) * inv
    tn = max(np.max(np.minimum(t0, t1)), tmin)
    return tn <= min(np.min(np.maximum(t0, t1)) * 1.001953125, btc), tn


def sph(c, rr, o, d, tmin):
    oc = o - c
    a, b, cc = d @ d, d @ oc, oc @ oc - rr
    disc = b * b - a * cc
    if disc <= 0:
        return None
    sq = np.sqrt(disc)
    tn, tf = (-b - sq) / a, (-b + sq) / a
    t = tn if tn > tmin else tf
    return t if tmin < t < 3.4e38 else None


def trace(o, d, time, tmin=0.001):
    ow = o + tshift
    with np.errstate(divide="ignore"):
        inv = np.clip(1.0 / d, -2.0 ** 64, 2.0 ** 64)
    best, btc = (np.inf, None), 3.4e38
    stack, cur, inner, leaf, tests = [NONE], root, 0, 0, 0
    while True:
        i, nxt = cur & 0x7FFF, NONE
        if not (cur & LEAF):
            inner += 1
            hits = []
            for q in range(4):
                lo = np.array([F[i, q], F[i, 8 + q], F[i, 16 + q]])
                hi = np.array([F[i, 4 + q], F[i, 12 + q], F[i, 20 + q]])
                with np.errstate(invalid="ignore"):
                    h, tn = slab(lo, hi, ow, inv, tmin, btc)
                if h:
                    hits.append((tn, int(R[i, q])))
            hits.sort()
            stack += [r for _, r in reversed(hits[1:])]
            if hits:
                nxt = hits[0][1]
        else:
            leaf += 1
            for q in range(4):
                r = int(R[i, q])
                if (r >> 28) == 15:
                    break
                tests += 1
                t = sph(F[i, 4 * q:4 * q + 3] + time * F[i, 16 + 3 * q:19 + 3 * q], F[i, 4 * q + 3], o, d, tmin)
                if t is not None and t < best[0]:
                    best, btc = (t, r & 0xFFFFFFF), t * (1 + 2 ** -9)
        if nxt == NONE:
            nxt = stack.pop() if len(stack) > 1 else NONE
        if nxt == NONE:
            return best, (inner, leaf, tests)
        cur = nxt


def brute(o, d, time, tmin=0.001):
    best = (np.inf, None)
    for j in range(nsph):
        t = sph(SF[j, 0:3] + time * SF[j, 4:7], SF[j, 3] * SF[j, 3], o, d, tmin)
        if t is not None and t < best[0]:
            best = (t, j)
    return best


scene = rtow.Scene.build("random_ned", n=487, image="synthetic", scene_seed=1)
W, H = 1920, 1080
cam, p = rtow.camera_main(W, H), rtow.params(W, H, 4, seed=1)
ocam, op = sio.RtowCamera.from_buffer_copy(bytes(cam)), sio.RtowParams.from_buffer_copy(bytes(p))
org, shift = np.array(cam.origin[:], np.float64), np.array([0.0, 0.0, 1000.0])  # the root Translate
rng = np.random.default_rng(3)
tot, rays, bad = np.zeros(3), 0, 0
for _ in range(npx):
    rec = sio.oracle_trace(scene.view_ptr, ocam, op, int(rng.integers(W)), int(rng.integers(H)), 0)
    prev = org.copy()
    for r in rec:
        pt = r[3:6].astype(np.float64)
        d = (pt - prev) / float(r[2]) if r[0] == 1.0 else pt
        (t, leaf_ref), st = trace(prev - shift, d, 0.5)
        bt, bi = brute(prev - shift, d, 0.5)
        bad += (leaf_ref is None) != (bi is None) or (bi is not None and abs(t - bt) > 1e-6 * max(1.0, bt))
        tot += st
        rays += 1
        if r[0] == 1.0:
            prev = pt
print(f"k={k}: {n} nodes, stack need {need}; {rays} segments of {npx} paths: inner steps {tot[0] / rays:.2f}, "
      f"leaf steps {tot[1] / rays:.2f}, sphere tests {tot[2] / rays:.2f} per ray; closest-hit mismatches {bad}")
