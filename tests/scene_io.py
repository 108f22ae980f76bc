"""Test helpers: RTOWSCN1 scene files, the synthetic texture, the C oracle.

The oracle (oracle/librtow_oracle.so) is test infrastructure: tests use it as
the checker only (see oracle/rtow_oracle.h).
"""
import ctypes
import json
import os
import struct

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE_SO = os.path.join(REPO, "oracle", "librtow_oracle.so")

HITABLE = np.dtype([("kind", "<u4"), ("a", "<u4"), ("b", "<u4"), ("c", "<u4"), ("f", "<f4", 12)])
MATERIAL = np.dtype([("kind", "<u4"), ("texture", "<u4"), ("param", "<f4"), ("albedo", "<f4", 3),
                     ("pad", "<u4", 2)])
TEXTURE = np.dtype([("kind", "<u4"), ("a", "<u4"), ("b", "<u4"), ("c", "<u4"), ("f", "<f4", 4)])
IMAGE = np.dtype([("nx", "<u4"), ("ny", "<u4"), ("channels", "<u4"), ("pad", "<u4"), ("offset", "<u8")])
PERLIN = np.dtype([("ranfloat", "<f4", 256), ("ranvec", "<f4", (256, 3)), ("perm_x", "<i4", 256),
                   ("perm_y", "<i4", 256), ("perm_z", "<i4", 256)])
assert HITABLE.itemsize == 64 and MATERIAL.itemsize == 32 and TEXTURE.itemsize == 32
assert IMAGE.itemsize == 24 and PERLIN.itemsize == 7168


def synthetic_image(nx, ny):
    """The synthetic stand-in for the 2048x1024 earth texture:
    r = 255*i/(nx-1), g = 255*j/(ny-1), b = 40 + 160*checker32(i,j) + (i*j & 31)."""
    i = np.arange(nx, dtype=np.int64)[None, :]
    j = np.arange(ny, dtype=np.int64)[:, None]
    r = (i * 255) // max(nx - 1, 1) + 0 * j
    g = (j * 255) // max(ny - 1, 1) + 0 * i
    b = 40 + 160 * (((i >> 5) + (j >> 5)) & 1) + ((i * j) & 31)
    return np.stack([r, g, b], axis=-1).astype(np.uint8)


def parse_scene(blob):
    """RTOWSCN1 bytes -> dict of numpy arrays (texels may be stripped)."""
    assert blob[:8] == b"RTOWSCN1", "not a scene file"
    hdr = struct.unpack("<10I", blob[8:48])
    (ntex,) = struct.unpack("<Q", blob[48:56])
    off = 56
    out = {"version": hdr[0], "root": hdr[1]}

    def take(dtype, count):
        nonlocal off
        a = np.frombuffer(blob, dtype=dtype, count=count, offset=off).copy()
        off += dtype.itemsize * count
        return a

    out["hitables"] = take(HITABLE, hdr[2])
    out["refs"] = take(np.dtype("<u4"), hdr[3])
    out["materials"] = take(MATERIAL, hdr[4])
    out["textures"] = take(TEXTURE, hdr[5])
    out["perlin"] = take(PERLIN, 1)[0] if hdr[7] else None
    out["images"] = take(IMAGE, hdr[6])
    out["texels"] = np.frombuffer(blob, dtype=np.uint8, count=ntex, offset=off).copy()
    off += ntex
    assert off == len(blob), "trailing bytes in scene file"
    return out


def load_scene(path):
    with open(path, "rb") as f:
        return parse_scene(f.read())


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_case(name):
    for c in manifest()["cases"]:
        if c["name"] == name:
            return c
    raise KeyError(name)


def golden_image(name, W, H):
    lin = np.fromfile(os.path.join(GOLDEN, name + ".lin"), dtype=np.float32).reshape(H, W, 3)
    bgra = np.fromfile(os.path.join(GOLDEN, name + ".bgra"), dtype=np.uint8).reshape(H, W, 4)
    return lin, bgra


# ---- ctypes mirror of include/rtow.h structs --------------------------------
class RtowScene(ctypes.Structure):
    _fields_ = [("root", ctypes.c_uint32), ("n_hitables", ctypes.c_uint32), ("hitables", ctypes.c_void_p),
                ("n_refs", ctypes.c_uint32), ("refs", ctypes.c_void_p), ("n_materials", ctypes.c_uint32),
                ("materials", ctypes.c_void_p), ("n_textures", ctypes.c_uint32), ("textures", ctypes.c_void_p),
                ("perlin", ctypes.c_void_p), ("n_images", ctypes.c_uint32), ("images", ctypes.c_void_p),
                ("n_texel_bytes", ctypes.c_uint64), ("texels", ctypes.c_void_p)]


class RtowCamera(ctypes.Structure):
    _fields_ = [("origin", ctypes.c_float * 3), ("lower_left_corner", ctypes.c_float * 3),
                ("horizontal", ctypes.c_float * 3), ("vertical", ctypes.c_float * 3), ("u", ctypes.c_float * 3),
                ("v", ctypes.c_float * 3), ("w", ctypes.c_float * 3), ("lens_radius", ctypes.c_float),
                ("time0", ctypes.c_float), ("time1", ctypes.c_float)]


class RtowParams(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("spp", ctypes.c_uint32),
                ("max_depth", ctypes.c_uint32), ("gi_enable", ctypes.c_uint32), ("sky_gain", ctypes.c_float),
                ("gi_gain", ctypes.c_float), ("samples_per_chunk", ctypes.c_uint32), ("seed", ctypes.c_uint64),
                ("rank", ctypes.c_uint32), ("world", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("blocks_per_cu", ctypes.c_uint32)]


class OracleCounters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "samples", "segments", "bvh_visits", "bvh_box_pass", "sphere_tests", "moving_sphere_tests",
        "rect_tests", "medium_calls", "list_visits", "draws", "max_draws_per_sample")]


def camera_from_file(path):
    cam = RtowCamera()
    data = open(path, "rb").read()
    assert len(data) == ctypes.sizeof(RtowCamera)
    ctypes.memmove(ctypes.addressof(cam), data, len(data))
    return cam


def default_params(W, H, spp, seed=1):
    return RtowParams(width=W, height=H, spp=spp, max_depth=50, gi_enable=1, sky_gain=1.0, gi_gain=0.3,
                      samples_per_chunk=0, seed=seed, rank=0, world=1, flags=0, blocks_per_cu=0)


class SceneArrays:
    """Keeps numpy arrays alive behind an RtowScene view."""

    def __init__(self, d):
        self.d = d
        self.perlin = np.array([d["perlin"]], dtype=PERLIN) if d["perlin"] is not None else None
        self.view = RtowScene(
            root=d["root"], n_hitables=len(d["hitables"]), hitables=d["hitables"].ctypes.data,
            n_refs=len(d["refs"]), refs=d["refs"].ctypes.data if len(d["refs"]) else None,
            n_materials=len(d["materials"]), materials=d["materials"].ctypes.data,
            n_textures=len(d["textures"]), textures=d["textures"].ctypes.data,
            perlin=self.perlin.ctypes.data if self.perlin is not None else None,
            n_images=len(d["images"]), images=d["images"].ctypes.data if len(d["images"]) else None,
            n_texel_bytes=len(d["texels"]), texels=d["texels"].ctypes.data if len(d["texels"]) else None)


def with_synthetic_texels(d):
    """Re-attach the synthetic texture's texels to a stripped golden scene."""
    if len(d["images"]) == 0 or len(d["texels"]):
        return d
    parts = []
    off = 0
    imgs = d["images"].copy()
    for k, im in enumerate(imgs):
        rgb = synthetic_image(int(im["nx"]), int(im["ny"])).reshape(-1)
        imgs[k]["offset"] = off
        parts.append(rgb)
        off += rgb.size
    d = dict(d)
    d["images"] = imgs
    d["texels"] = np.concatenate(parts)
    return d


_oracle = None


def oracle():
    global _oracle
    if _oracle is None:
        lib = ctypes.CDLL(ORACLE_SO)
        lib.rtow_oracle_render_pixels.argtypes = [ctypes.c_void_p, ctypes.POINTER(RtowCamera),
                                                  ctypes.POINTER(RtowParams), ctypes.c_void_p, ctypes.c_uint32,
                                                  ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.POINTER(OracleCounters)]
        lib.rtow_oracle_render_pixels.restype = ctypes.c_int
        lib.rtow_oracle_trace_sample.argtypes = [ctypes.c_void_p, ctypes.POINTER(RtowCamera),
                                                 ctypes.POINTER(RtowParams), ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]
        lib.rtow_oracle_trace_sample.restype = ctypes.c_int
        _oracle = lib
    return _oracle


def oracle_trace(scene_view_ptr, cam, params, x, y, sample, max_segments=64):
    """The oracle's path of one sample: [n, 12] float32 segment records."""
    lib = oracle()
    out = np.zeros((max_segments, 12), np.float32)
    n = ctypes.c_uint32()
    rc = lib.rtow_oracle_trace_sample(scene_view_ptr, ctypes.byref(cam), ctypes.byref(params), x, y, sample,
                                      out.ctypes.data, max_segments, ctypes.byref(n))
    if rc != 0:
        raise RuntimeError(f"oracle trace failed: {rc}")
    return out[: n.value]


def oracle_render(scene_view_ptr, cam, params, pixels=None, threads=None):
    """Render with the C oracle.  scene_view_ptr: address of an rtow_scene.
    Returns (lin [n,3] float32, bgra [n,4] uint8, counters)."""
    lib = oracle()
    if pixels is None:
        n = params.width * params.height
        pix_ptr = None
    else:
        pixels = np.ascontiguousarray(pixels, dtype=np.uint32)
        n = pixels.size
        pix_ptr = pixels.ctypes.data
    lin = np.zeros((n, 3), np.float32)
    bgra = np.zeros((n, 4), np.uint8)
    c = OracleCounters()
    threads = threads or min(8, os.cpu_count() or 1)
    rc = lib.rtow_oracle_render_pixels(scene_view_ptr, ctypes.byref(cam), ctypes.byref(params), pix_ptr, n,
                                       threads, lin.ctypes.data, bgra.ctypes.data, ctypes.byref(c))
    if rc != 0:
        raise RuntimeError(f"oracle render failed: {rc}")
    return lin, bgra, c


def rms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)))


# ---- editing flattened scenes (tie / edge-case tests) ----------------------
HIT_SPHERE, HIT_MOVING_SPHERE, HIT_TRANSLATE, HIT_LIST, HIT_BVH_NODE = 1, 2, 7, 9, 11


def scene_check(scene):
    """rtow_scene_check on any object with a view_ptr: (stack_need, chain_need)."""
    import rtow

    sn, cn = ctypes.c_uint32(), ctypes.c_uint32()
    rtow.check(rtow.lib().rtow_scene_check(scene.view_ptr, ctypes.byref(sn), ctypes.byref(cn)), "rtow_scene_check")
    return sn.value, cn.value


def scene_dict(scene):
    """A library-owned rtow.Scene as a dict of numpy arrays (via RTOWSCN1)."""
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "s.scn")
        scene.save(p)
        return load_scene(p)


def hitable_box(h, i):
    """Bounding box of hitable i the way the reference computes it
    (sphere.h:71-74, 120-127; bvhNode.h:58 union of the children)."""
    e = h[i]
    if e["kind"] == HIT_SPHERE:
        c, r = e["f"][:3].astype(np.float32), np.float32(e["f"][3])
        return c - r, c + r
    if e["kind"] == HIT_MOVING_SPHERE:
        c0, c1, r = e["f"][:3], e["f"][3:6], np.float32(e["f"][8])
        return np.minimum(c0, c1) - r, np.maximum(c0, c1) + r
    if e["kind"] == HIT_BVH_NODE:
        a0, a1 = hitable_box(h, e["a"])
        b0, b1 = hitable_box(h, e["b"])
        return np.minimum(a0, b0), np.maximum(a1, b1)
    raise ValueError(f"no box for kind {e['kind']}")


def refresh_bvh_boxes(d):
    """Recompute every BvhNode's stored box from its children (after moving
    leaves), bottom-up, in place."""
    h = d["hitables"]
    for i in range(len(h)):
        if h[i]["kind"] == HIT_BVH_NODE:
            lo, hi = hitable_box(h, i)
            h[i]["f"][:3] = lo
            h[i]["f"][3:6] = hi


def bvh_leaves_in_order(d):
    """Hitable indices of the leaves under the root's BvhNode, left to right."""
    h = d["hitables"]
    i = d["root"]
    while h[i]["kind"] == HIT_TRANSLATE:
        i = h[i]["a"]
    out = []

    def walk(k):
        if h[k]["kind"] == HIT_BVH_NODE:
            walk(h[k]["a"])
            if h[k]["b"] != h[k]["a"]:
                walk(h[k]["b"])
        else:
            out.append(int(k))

    walk(i)
    return out


class ArrayScene:
    """An edited scene dict behind the `view_ptr` interface rtow.Context.upload
    and oracle_render take."""

    def __init__(self, d):
        self.arrays = SceneArrays(d)

    @property
    def view_ptr(self):
        return ctypes.addressof(self.arrays.view)


def tie_scene(n=100):
    """random_ned with an exact duplicate of a large sphere: leaf X (earlier in
    the reference tree's left-to-right order) is moved onto leaf Y's center and
    radius, boxes refreshed.  Every ray that meets one meets both at the same
    t; BvhNode::hit (bvhNode.h:74-77) hands the tie to the later leaf.
    Returns (dict, earlier leaf, later leaf)."""
    import rtow

    d = scene_dict(rtow.Scene.build("random_ned", n=n, image="none"))
    h = d["hitables"]
    leaves = bvh_leaves_in_order(d)
    big = [k for k in leaves if h[k]["kind"] == HIT_SPHERE and 0.45 < h[k]["f"][3] < 10]
    small = [k for k in leaves if h[k]["kind"] == HIT_SPHERE and h[k]["f"][3] < 0.3]
    # Y: the large sphere nearest the main camera among those on screen
    cam = rtow.camera_main(64, 36)
    org, llc = np.array(cam.origin[:]), np.array(cam.lower_left_corner[:])
    hor, ver = np.array(cam.horizontal[:]), np.array(cam.vertical[:])
    off = h[d["root"]]["f"][:3] if h[d["root"]]["kind"] == HIT_TRANSLATE else np.zeros(3)

    def screen(k):
        c = h[k]["f"][:3].astype(np.float64) + off
        u, v, s = np.linalg.solve(np.stack([hor, ver, -(c - org)], axis=1), org - llc)
        return u, v, np.linalg.norm(c - org)

    on = [(screen(k)[2], k) for k in big if all(0.15 < q < 0.85 for q in screen(k)[:2])]
    y = min(on)[1]
    x = small[-1] if leaves.index(small[-1]) > leaves.index(y) else small[0]
    h[x]["f"][:4] = h[y]["f"][:4]
    refresh_bvh_boxes(d)
    pos = {k: leaves.index(k) for k in (x, y)}
    early, late = sorted((x, y), key=lambda k: pos[k])
    return d, early, late


# ---- scene-graph edits (tests build reference-legal worlds the fixtures do not hold)
def copy_scene(d):
    return {k: (v.copy() if hasattr(v, "copy") else v) for k, v in d.items()}


def with_items(d, lst, items):
    """A copy of d whose list hitable `lst` holds `items` (appended refs)."""
    e = copy_scene(d)
    e["hitables"][lst]["a"] = len(e["refs"])
    e["hitables"][lst]["b"] = len(items)
    e["refs"] = np.concatenate([e["refs"], np.array(items, np.uint32)])
    return e


def add_list(d, members):
    """Append a HitableList hitable over `members`; returns (dict, its index)."""
    e = copy_scene(d)
    h = np.zeros(1, dtype=HITABLE)
    h[0]["kind"] = HIT_LIST
    h[0]["a"] = len(e["refs"])
    h[0]["b"] = len(members)
    e["refs"] = np.concatenate([e["refs"], np.array(members, np.uint32)])
    e["hitables"] = np.concatenate([e["hitables"], h])
    return e, len(e["hitables"]) - 1


def bvh_leaves(h, i):
    """The leaves of BvhNode i in left-to-right order (an n == 1 node once)."""
    if h[i]["kind"] == HIT_BVH_NODE:
        out = bvh_leaves(h, h[i]["a"])
        if h[i]["b"] != h[i]["a"]:
            out += bvh_leaves(h, h[i]["b"])
        return out
    return [int(i)]
