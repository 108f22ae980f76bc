#!/usr/bin/env python3
"""Golden fixture for residual corner (i), from the REFERENCE ITSELF
(oracle/_ref/ref_harness `graze_medium`, the reference's own classes):

one exact primary ray -- pixel (COL, ROW), sample SAMPLE of a WxH frame,
computed by the oracle (rtow_oracle_camera_ray, the render loop's own float
arithmetic) -- grazes the y-min edge of a Box's x-min side.  The Box sits in
an n == 1 BvhNode; the side x = k is placed where the ray crosses that plane
(t_k = (k - o.x) / d.x, y_k = o.y + t_k d.y: the rectangle test's own
arithmetic, so y_k lies exactly on the edge and the closed bounds of
xy_rect.h accept it), and k is searched until AABB::hit (aabb.h:22-43) sees
the ray leave the y slab no later than it enters the x slab: `tmax <= tmin`,
the Box is never tested.  Behind the BvhNode in the list: a ConstantMedium
(sphere boundary 3 units beyond the edge point), then a sphere 3 units in
front of it, which the ray hits first.  The reference asks the medium with
the whole interval and draws its scatter distance; a traversal that took the
grazed side hands the medium that side's t, skips that draw and ends at the
same sphere one draw behind -- every later bounce of the sample differs.

Writes graze_medium.{scn,lin,bgra,params} and adds the case to
manifest_extra.json (`trace`: the sample).
Usage: python3 tests/golden/make_graze_golden.py   (after make -C oracle ref)
"""
import ctypes
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(REPO, "ray-tracing-one-weekend_amd")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402
from make_golden import strip_texels  # noqa: E402

W, H, SPP, SEED = 24, 16, 4, 21
COL, ROW, SAMPLE = 5, 9, 0
f32 = np.float32


def primary_ray():
    cam = sio.RtowCamera.from_buffer_copy(bytes(rtow.camera_main(W, H)))
    p = sio.default_params(W, H, SPP, seed=SEED)
    out = (ctypes.c_float * 7)()
    lib = sio.oracle()
    lib.rtow_oracle_camera_ray.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.c_void_p]
    assert lib.rtow_oracle_camera_ray(ctypes.byref(cam), ctypes.byref(p), COL, ROW, SAMPLE, out) == 0
    v = np.array(out[:], np.float32)
    return v[:3], v[3:6]


def grazes(o, d, k):
    """float32 arithmetic of the rectangle test and of AABB::hit for the Box
    [k, k+1] x [y_k, y_k+1] x [z_k-1, z_k+1]: (y_k, z_k, box, skipped?)."""
    tk = (f32(k) - o[0]) / d[0]
    yk = o[1] + tk * d[1]
    zk = o[2] + tk * d[2]
    lo = np.array([k, yk, zk - f32(1)], np.float32)
    hi = np.array([f32(k) + f32(1), yk + f32(1), zk + f32(1)], np.float32)
    tmin, tmax = f32(0.001), f32(np.finfo(np.float32).max)
    for a in range(3):
        p = (lo[a] - o[a]) / d[a]
        q = (hi[a] - o[a]) / d[a]
        t0 = p if p < q else q
        t1 = p if p > q else q
        tmin = t0 if t0 > tmin else tmin
        tmax = t1 if t1 < tmax else tmax
        if tmax <= tmin:
            return yk, zk, lo, hi, True
    return yk, zk, lo, hi, False


def main():
    if not os.access(HARNESS, os.X_OK):
        sys.exit("build the harness first: make -C oracle ref")
    o, d = primary_ray()
    assert d[0] > 0 and d[1] < 0, (o, d)
    found = None
    for i in range(20000):
        k = f32(8.0) + f32(i) * f32(0.0009765625)
        yk, zk, lo, hi, skipped = grazes(o, d, k)
        if skipped:
            found = (k, yk, zk, lo, hi)
            break
    assert found, "no grazing plane found"
    k, yk, zk, lo, hi = found
    dn = d.astype(np.float64) / np.linalg.norm(d.astype(np.float64))
    tk = (np.float64(f32(k) - o[0]) / np.float64(d[0]))
    pt = o.astype(np.float64) + tk * d.astype(np.float64)
    med = (pt + 3.0 * dn).astype(np.float32)
    sph = (pt - 3.0 * dn).astype(np.float32)
    params = [*lo, *hi, *med, f32(1.0), *sph, f32(0.5)]
    tmp = tempfile.mkdtemp(prefix="rtow_graze_")
    ppath = os.path.join(HERE, "graze_medium.params")
    with open(ppath, "w") as fh:
        fh.write(" ".join(float(v).hex() for v in params) + "\n")
    env = dict(os.environ, RTOW_SCENE_SEED="1", RTOW_GRAZE_PARAMS=ppath)
    raw = os.path.join(tmp, "graze_medium.scn")
    subprocess.run([HARNESS, "dump", "graze_medium", raw, "--cwd", tmp], env=env, check=True, capture_output=True)
    sha, ntex, hdr = strip_texels(raw, os.path.join(HERE, "graze_medium.scn"))
    subprocess.run([HARNESS, "render", "graze_medium", str(W), str(H), str(SPP), os.path.join(HERE, "graze_medium"),
                    "--seed", str(SEED), "--cwd", tmp], env=env, check=True)
    subprocess.run([HARNESS, "camera", str(W), str(H), os.path.join(HERE, f"cam_{W}x{H}.cam")], env=env, check=True)
    mpath = os.path.join(HERE, "manifest_extra.json")
    m = json.load(open(mpath))
    m["cases"] = [c for c in m["cases"] if c["name"] != "graze_medium"]
    m["cases"].append(dict(name="graze_medium", harness="ref_harness", flags=0, scene="graze_medium", n=0,
                           image="none", width=W, height=H, spp=SPP, seed=SEED, texel_bytes=ntex, texel_sha256=sha,
                           n_hitables=hdr[2], trace=[COL, ROW, SAMPLE], plane_k=float(k)))
    with open(mpath, "w") as fh:
        json.dump(m, fh, indent=1)
    print(f"graze_medium: k = {float(k)!r}, {hdr[2]} hitables")


if __name__ == "__main__":
    main()
