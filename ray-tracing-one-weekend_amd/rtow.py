"""Python mirror of the C-ABI (include/rtow.h) over librtow_hip.so.

Host-side plumbing for tests, bench.py and __graft_entry__: build a scene the
way scenes.h does, upload it, render on the GPU.  The rendering itself is the
HIP path in librtow_hip.so; there is no Python or CPU fallback -- if the
library is missing this module raises.
"""
import ctypes
import os
import re

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
LIB_PATH = os.environ.get("RTOW_LIB") or os.path.join(PKG_DIR, "librtow_hip.so")
HEADER = os.path.join(REPO, "include", "rtow.h")

# ---- constants (include/rtow.h) ---------------------------------------------
OK, E_INVALID, E_UNSUPPORTED, E_HIP, E_NO_DEVICE, E_IO, E_NOMEM, E_RCCL = 0, -1, -2, -3, -4, -5, -6, -7
SCENE_THREE_SPHERE, SCENE_RANDOM_NED, SCENE_CORNELL_NED, SCENE_CORNELL_SMOKE = 1, 2, 3, 4
SCENE_FINAL_NED, SCENE_RANDOM, SCENE_CORNELL = 5, 6, 7
SCENES = {"three_sphere": SCENE_THREE_SPHERE, "random_ned": SCENE_RANDOM_NED, "cornell": SCENE_CORNELL_NED,
          "cornell_smoke": SCENE_CORNELL_SMOKE, "final_ned": SCENE_FINAL_NED,
          "random": SCENE_RANDOM, "cornell_box": SCENE_CORNELL}  # (the last two: scenes.h's non-NED builders)
IMAGE_NONE, IMAGE_SYNTHETIC, IMAGE_RAW, IMAGE_JPEG = 0, 1, 2, 3
IMAGES = {"none": IMAGE_NONE, "synthetic": IMAGE_SYNTHETIC, "raw": IMAGE_RAW, "jpeg": IMAGE_JPEG}
FLAG_STATS = 1


class Scene_(ctypes.Structure):
    _fields_ = [("root", ctypes.c_uint32), ("n_hitables", ctypes.c_uint32), ("hitables", ctypes.c_void_p),
                ("n_refs", ctypes.c_uint32), ("refs", ctypes.c_void_p), ("n_materials", ctypes.c_uint32),
                ("materials", ctypes.c_void_p), ("n_textures", ctypes.c_uint32), ("textures", ctypes.c_void_p),
                ("perlin", ctypes.c_void_p), ("n_images", ctypes.c_uint32), ("images", ctypes.c_void_p),
                ("n_texel_bytes", ctypes.c_uint64), ("texels", ctypes.c_void_p)]


class Camera(ctypes.Structure):
    _fields_ = [("origin", ctypes.c_float * 3), ("lower_left_corner", ctypes.c_float * 3),
                ("horizontal", ctypes.c_float * 3), ("vertical", ctypes.c_float * 3), ("u", ctypes.c_float * 3),
                ("v", ctypes.c_float * 3), ("w", ctypes.c_float * 3), ("lens_radius", ctypes.c_float),
                ("time0", ctypes.c_float), ("time1", ctypes.c_float)]


class Params(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("spp", ctypes.c_uint32),
                ("max_depth", ctypes.c_uint32), ("gi_enable", ctypes.c_uint32), ("sky_gain", ctypes.c_float),
                ("gi_gain", ctypes.c_float), ("samples_per_chunk", ctypes.c_uint32), ("seed", ctypes.c_uint64),
                ("rank", ctypes.c_uint32), ("world", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("blocks_per_cu", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("segments", ctypes.c_uint64), ("samples", ctypes.c_uint64), ("pixels", ctypes.c_uint64),
                ("kernel_ms", ctypes.c_double), ("resolve_ms", ctypes.c_double), ("total_ms", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Plan(ctypes.Structure):
    _fields_ = [("samples_per_chunk", ctypes.c_uint32), ("n_big", ctypes.c_uint32),
                ("tail_samples", ctypes.c_uint32), ("n_tail", ctypes.c_uint32), ("n_chunks", ctypes.c_uint32),
                ("n_local_px", ctypes.c_uint32), ("n_items", ctypes.c_uint64), ("cus", ctypes.c_uint32),
                ("pad", ctypes.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "pad"}


class BuildOpts(ctypes.Structure):
    _fields_ = [("scene_seed", ctypes.c_uint64), ("n", ctypes.c_uint32), ("image_mode", ctypes.c_uint32),
                ("image_path", ctypes.c_char_p), ("image_nx", ctypes.c_uint32), ("image_ny", ctypes.c_uint32),
                ("wrap_world", ctypes.c_uint32), ("ground_side", ctypes.c_uint32)]


class RtowError(RuntimeError):
    def __init__(self, code, where, detail):
        super().__init__(f"{where} failed: {code} ({detail})")
        self.code = code


_lib = None


def lib():
    """Load librtow_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it first (python -c 'import __graft_entry__ as g; g.build()')")
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    sig = {
        "rtow_abi_version": ([], i32),
        "rtow_error_string": ([i32], ctypes.c_char_p),
        "rtow_last_error": ([], ctypes.c_char_p),
        "rtow_params_default": ([ctypes.POINTER(Params), u32, u32, u32], None),
        "rtow_tile_count": ([u32, u32], u32),
        "rtow_rank_tile_count": ([u32, u32, u32, u32], u32),
        "rtow_build_opts_default": ([ctypes.POINTER(BuildOpts)], None),
        "rtow_build_scene": ([i32, ctypes.POINTER(BuildOpts), ctypes.POINTER(vp)], i32),
        "rtow_scene_view": ([vp], vp),
        "rtow_scene_free": ([vp], None),
        "rtow_scene_save": ([vp, ctypes.c_char_p], i32),
        "rtow_scene_load": ([ctypes.c_char_p, ctypes.POINTER(vp)], i32),
        "rtow_scene_draws": ([vp], u32),
        "rtow_scene_check": ([vp, ctypes.POINTER(u32), ctypes.POINTER(u32)], i32),
        "rtow_camera_main": ([u32, u32, ctypes.POINTER(Camera)], i32),
        "rtow_camera_oriented": ([u32, u32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                  ctypes.POINTER(Camera)], i32),
        "rtow_camera_look_at": ([ctypes.POINTER(ctypes.c_float)] * 3 + [ctypes.c_float] * 6 + [ctypes.POINTER(Camera)],
                                i32),
        "rtow_render_progressive": ([vp, ctypes.POINTER(Camera), ctypes.POINTER(Params), i32, vp, vp,
                                     ctypes.POINTER(u32), ctypes.POINTER(Stats)], i32),
        "rtow_synthetic_image": ([u32, u32, vp], None),
        "rtow_device_count": ([ctypes.POINTER(i32)], i32),
        "rtow_context_create": ([i32, ctypes.POINTER(vp)], i32),
        "rtow_context_destroy": ([vp], i32),
        "rtow_scene_upload": ([vp, vp], i32),
        "rtow_context_set_tree": ([vp, i32], i32),
        "rtow_render_plan": ([vp, ctypes.POINTER(Params), ctypes.POINTER(Plan)], i32),
        "rtow_debug_trace_sample": ([vp, ctypes.POINTER(Camera), ctypes.POINTER(Params), u32, u32, u32, vp, u32,
                                     ctypes.POINTER(u32)], i32),
        "rtow_write_bmp": ([ctypes.c_char_p, vp, ctypes.c_uint64, u32, u32, u32], i32),
        "rtow_write_ppm": ([ctypes.c_char_p, vp, u32, u32], i32),
        "rtow_render": ([vp, ctypes.POINTER(Camera), ctypes.POINTER(Params), vp, vp, ctypes.POINTER(Stats)], i32),
        "rtow_render_tiles_device": ([vp, ctypes.POINTER(Camera), ctypes.POINTER(Params), vp, vp, vp,
                                      ctypes.POINTER(Stats)], i32),
        "rtow_render_progressive_tiles_device": ([vp, ctypes.POINTER(Camera), ctypes.POINTER(Params), i32, vp, vp,
                                                  vp, ctypes.POINTER(u32), ctypes.POINTER(Stats)], i32),
        "rtow_assemble_device": ([vp, u32, u32, u32, vp, u32, vp, vp], i32),
        "rtow_assemble_linear_device": ([vp, u32, u32, u32, vp, u32, vp, vp], i32),
        "rtow_multi_create": ([ctypes.POINTER(i32), u32, ctypes.POINTER(vp)], i32),
        "rtow_multi_destroy": ([vp], i32),
        "rtow_multi_device_count": ([vp], u32),
        "rtow_multi_set_tree": ([vp, i32], i32),
        "rtow_multi_upload": ([vp, vp], i32),
        "rtow_multi_render": ([vp, ctypes.POINTER(Camera), ctypes.POINTER(Params), vp, vp, ctypes.POINTER(Stats),
                               vp], i32),
        "rtow_render_devices": ([ctypes.POINTER(i32), u32, vp, ctypes.POINTER(Camera), ctypes.POINTER(Params), vp, vp,
                                 ctypes.POINTER(Stats)], i32),
        "rtow_image_decode_jpeg": ([ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(vp), ctypes.POINTER(u32),
                                    ctypes.POINTER(u32), ctypes.POINTER(u32)], i32),
        "rtow_image_load_jpeg": ([ctypes.c_char_p, ctypes.POINTER(vp), ctypes.POINTER(u32), ctypes.POINTER(u32),
                                  ctypes.POINTER(u32)], i32),
        "rtow_image_free": ([vp], None),
    }
    for name, (args, res) in sig.items():
        if not hasattr(L, name) and os.environ.get("RTOW_LIB"):
            continue  # an older build loaded for A/B comparison (tools/ab.py)
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def source_hash():
    """sha256 (first 16 hex digits) of everything librtow_hip.so is compiled
    from: the device/host sources, the headers and the Makefile (its flags).
    A PMC summary under profiles/ records the hash of the build it measured,
    so bench.py can tell whether those counters describe the kernel it runs."""
    import hashlib

    files = [os.path.join(PKG_DIR, "Makefile")]
    csrc = os.path.join(PKG_DIR, "csrc")
    files += [os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".cpp", ".h"))]
    files += [os.path.join(REPO, "include", f) for f in ("rtow.h", "rtow_rng.h")]  # not rtow_reference.hpp
    h = hashlib.sha256()
    for f in sorted(files, key=lambda p: os.path.relpath(p, REPO)):
        h.update(os.path.relpath(f, REPO).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def host_threads():
    """(threads, info): the host threads this process may use -- the CPUs in
    its affinity mask, capped by a cgroup v2 CPU quota when one is set (a GPU
    box shares one machine's CPUs between its GPUs) -- and a dict naming the
    machine's CPU count, the affinity, the quota and the CPU model."""
    import math

    machine = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = machine
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    threads = affinity if quota is None else max(1, min(affinity, math.ceil(quota)))
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return threads, {"machine_cpus": machine, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
                     "cpu_model": model}


def header_functions():
    """Names of the functions include/rtow.h declares."""
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rtow_[a-z0-9_]+)\s*\(", text)))


def check(rc, where):
    if rc != OK:
        L = lib()
        raise RtowError(rc, where, f"{L.rtow_error_string(rc).decode()}: {L.rtow_last_error().decode()}")


FLAG_STATS = 1 << 0
FLAG_CAMERA_DOF = 1 << 1  # CAMERA_DOF_EN 1 (camera.h:124-126)
FLAG_FRAME_PLAN = 1 << 2  # every rank chunks its samples as the whole frame does (rtow_render's sums)


def params(width, height, spp, seed=1, **kw):
    p = Params()
    lib().rtow_params_default(ctypes.byref(p), width, height, spp)
    p.seed = seed
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def camera_main(width, height):
    """The camera main.cpp:111-125 builds for a width x height frame."""
    c = Camera()
    check(lib().rtow_camera_main(width, height, ctypes.byref(c)), "rtow_camera_main")
    return c


def camera_look_at(look_from, look_at, up, vfov_deg, aspect, aperture, focus_distance, time0=0.0, time1=1.0):
    """Camera(...) with setCamera_Euler's look-at basis (camera.h:271-313)."""
    f3 = lambda v: (ctypes.c_float * 3)(*v)  # noqa: E731
    c = Camera()
    check(lib().rtow_camera_look_at(f3(look_from), f3(look_at), f3(up), vfov_deg, aspect, aperture, focus_distance,
                                    time0, time1, ctypes.byref(c)), "rtow_camera_look_at")
    return c


def camera_oriented(width, height, look_from, rows):
    """The main camera after setOrientationMatrix(rows view/east/down) + setLookFromPoint."""
    lf = (ctypes.c_float * 3)(*look_from)
    rw = (ctypes.c_float * 9)(*np.asarray(rows, np.float32).reshape(-1))
    c = Camera()
    check(lib().rtow_camera_oriented(width, height, lf, rw, ctypes.byref(c)), "rtow_camera_oriented")
    return c


def plan(p, ctx=None):
    """rtow_render_plan: how a render with params `p` cuts its work items (ctx
    None: a 256-CU MI355X)."""
    out = Plan()
    check(lib().rtow_render_plan(ctx._h if ctx is not None else None, ctypes.byref(p), ctypes.byref(out)),
          "rtow_render_plan")
    return out


def tile_count(width, height):
    return lib().rtow_tile_count(width, height)


def rank_tile_count(width, height, rank, world):
    return lib().rtow_rank_tile_count(width, height, rank, world)


def decode_jpeg(data):
    """JPEG bytes -> (H, W, C) uint8 array, as the reference's stbi_load(.., 0) returns it."""
    import numpy as np

    L = lib()
    px, nx, ny, ch = ctypes.c_void_p(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    check(L.rtow_image_decode_jpeg(bytes(data), len(data), ctypes.byref(px), ctypes.byref(nx), ctypes.byref(ny),
                                   ctypes.byref(ch)), "rtow_image_decode_jpeg")
    try:
        n = nx.value * ny.value * ch.value
        out = np.frombuffer(ctypes.string_at(px.value, n), dtype=np.uint8).reshape(ny.value, nx.value, ch.value)
        return out.copy()
    finally:
        L.rtow_image_free(px)


def synthetic_image(nx, ny):
    out = np.zeros((ny, nx, 3), np.uint8)
    lib().rtow_synthetic_image(nx, ny, out.ctypes.data)
    return out


def write_bmp(path, pixels, width, height, bits_per_pixel=32):
    """The reference's BMP writer (winDIBbitmap.cpp:20-168) on a frame buffer."""
    buf = np.ascontiguousarray(pixels, dtype=np.uint8)
    check(lib().rtow_write_bmp(path.encode(), buf.ctypes.data, buf.nbytes, width, height, bits_per_pixel),
          "rtow_write_bmp")


def write_ppm(path, bgra):
    """bgra: [H, W, 4] uint8 frame (top row first) -> binary PPM."""
    buf = np.ascontiguousarray(bgra, dtype=np.uint8)
    check(lib().rtow_write_ppm(path.encode(), buf.ctypes.data, buf.shape[1], buf.shape[0]), "rtow_write_ppm")


TREES = {"sah": 0, "reference": 1}


class Scene:
    """A flattened world (owned by the library)."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle)

    @classmethod
    def build(cls, scene="random_ned", n=100, image="synthetic", scene_seed=1, wrap_world=True, image_path=None,
              image_size=(0, 0), ground_side=0):
        o = BuildOpts()
        lib().rtow_build_opts_default(ctypes.byref(o))
        o.scene_seed = scene_seed
        o.n = n
        o.image_mode = IMAGES[image]
        o.image_path = image_path.encode() if image_path else None
        o.image_nx, o.image_ny = image_size
        o.wrap_world = 1 if wrap_world else 0
        o.ground_side = ground_side
        h = ctypes.c_void_p()
        check(lib().rtow_build_scene(SCENES[scene], ctypes.byref(o), ctypes.byref(h)), "rtow_build_scene")
        return cls(h.value)

    @classmethod
    def load(cls, path):
        h = ctypes.c_void_p()
        check(lib().rtow_scene_load(path.encode(), ctypes.byref(h)), "rtow_scene_load")
        return cls(h.value)

    @property
    def view_ptr(self):
        return lib().rtow_scene_view(self._h)

    @property
    def view(self):
        return Scene_.from_address(self.view_ptr)

    @property
    def draws(self):
        return lib().rtow_scene_draws(self._h)

    def save(self, path):
        check(lib().rtow_scene_save(self.view_ptr, path.encode()), "rtow_scene_save")

    def check(self):
        sn, cn = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().rtow_scene_check(self.view_ptr, ctypes.byref(sn), ctypes.byref(cn)), "rtow_scene_check")
        return sn.value, cn.value

    def __del__(self):
        try:
            if self._h and _lib is not None:
                _lib.rtow_scene_free(self._h)
                self._h = None
        except Exception:
            pass


def device_count():
    n = ctypes.c_int(0)
    rc = lib().rtow_device_count(ctypes.byref(n))
    return n.value if rc == OK else 0


class Context:
    """One GPU: its stream, the uploaded scene and the work buffers."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        check(lib().rtow_context_create(device, ctypes.byref(h)), "rtow_context_create")
        self._h = h

    def set_tree(self, tree):
        """'sah' (default) or 'reference': the tree the next upload builds for
        BvhNode+sphere scenes (the frame is the same either way)."""
        check(lib().rtow_context_set_tree(self._h, TREES[tree]), "rtow_context_set_tree")

    def upload(self, scene):
        check(lib().rtow_scene_upload(self._h, scene.view_ptr), "rtow_scene_upload")

    def render(self, cam, p, linear=True):
        """rtow_render: returns (bgra[H,W,4] uint8, linear[H,W,3] float32 or None, Stats)."""
        bgra = np.zeros((p.height, p.width, 4), np.uint8)
        lin = np.zeros((p.height, p.width, 3), np.float32) if linear else None
        st = Stats()
        check(lib().rtow_render(self._h, ctypes.byref(cam), ctypes.byref(p), bgra.ctypes.data,
                                lin.ctypes.data if linear else None, ctypes.byref(st)), "rtow_render")
        return bgra, lin, st

    def render_progressive(self, cam, p, reset=False, linear=True):
        """rtow_render_progressive: p.spp new samples per pixel added to the running
        sums; returns (bgra, linear or None, total spp, Stats)."""
        bgra = np.zeros((p.height, p.width, 4), np.uint8)
        lin = np.zeros((p.height, p.width, 3), np.float32) if linear else None
        total = ctypes.c_uint32()
        st = Stats()
        check(lib().rtow_render_progressive(self._h, ctypes.byref(cam), ctypes.byref(p), 1 if reset else 0,
                                            bgra.ctypes.data, lin.ctypes.data if linear else None,
                                            ctypes.byref(total), ctypes.byref(st)), "rtow_render_progressive")
        return bgra, lin, total.value, st

    def trace_sample(self, cam, p, x, y, sample, max_segments=64):
        """rtow_debug_trace_sample: [n, 12] float32 segment records of one sample."""
        out = np.zeros((max_segments, 12), np.float32)
        n = ctypes.c_uint32()
        check(lib().rtow_debug_trace_sample(self._h, ctypes.byref(cam), ctypes.byref(p), x, y, sample, out.ctypes.data,
                                            max_segments, ctypes.byref(n)), "rtow_debug_trace_sample")
        return out[: n.value]

    def render_tiles_device(self, cam, p, d_bgra_slab, d_lin_slab=None, stream=None):
        """rtow_render_tiles_device on device pointers (ints); returns Stats."""
        st = Stats()
        check(lib().rtow_render_tiles_device(self._h, ctypes.byref(cam), ctypes.byref(p), d_bgra_slab, d_lin_slab,
                                             stream, ctypes.byref(st)), "rtow_render_tiles_device")
        return st

    def render_progressive_tiles_device(self, cam, p, d_bgra_slab, d_lin_slab=None, reset=False, stream=None):
        """rtow_render_progressive_tiles_device on device pointers (ints): p.spp new
        samples of rank p.rank's tiles added to the running sums, the average so far
        written to the slabs; returns (total spp, Stats)."""
        total = ctypes.c_uint32()
        st = Stats()
        check(lib().rtow_render_progressive_tiles_device(self._h, ctypes.byref(cam), ctypes.byref(p), 1 if reset else 0,
                                                         d_bgra_slab, d_lin_slab, stream, ctypes.byref(total),
                                                         ctypes.byref(st)), "rtow_render_progressive_tiles_device")
        return total.value, st

    def assemble_device(self, width, height, world, d_slabs, stride_px, d_frame, stream=None):
        check(lib().rtow_assemble_device(self._h, width, height, world, d_slabs, stride_px, d_frame, stream),
              "rtow_assemble_device")

    def assemble_linear_device(self, width, height, world, d_slabs, stride_px, d_frame, stream=None):
        check(lib().rtow_assemble_linear_device(self._h, width, height, world, d_slabs, stride_px, d_frame, stream),
              "rtow_assemble_linear_device")

    def close(self):
        if self._h:
            lib().rtow_context_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Multi:
    """rtow_multi: several GPUs from one process (entry i of `devices` renders
    rank i of n, one gather to the first device -- RCCL when the devices are
    distinct, device copies when one is listed more than once -- which
    assembles the frame; equal to rtow_render's frame bit for bit)."""

    def __init__(self, devices):
        devs = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        check(lib().rtow_multi_create(devs, len(devices), ctypes.byref(h)), "rtow_multi_create")
        self._h = h
        self.n = len(devices)

    def set_tree(self, tree):
        check(lib().rtow_multi_set_tree(self._h, TREES[tree]), "rtow_multi_set_tree")

    def upload(self, scene):
        check(lib().rtow_multi_upload(self._h, scene.view_ptr), "rtow_multi_upload")

    def render(self, cam, p, linear=True, host=True):
        """(bgra[H,W,4], linear[H,W,3] or None, Stats, [per-device Stats]).
        host=False: the frame stays on the first device (no copy out; bgra and
        linear are None), as bench.py --inproc times it."""
        bgra = np.zeros((p.height, p.width, 4), np.uint8) if host else None
        lin = np.zeros((p.height, p.width, 3), np.float32) if linear and host else None
        st = Stats()
        dst = (Stats * self.n)()
        check(lib().rtow_multi_render(self._h, ctypes.byref(cam), ctypes.byref(p),
                                      bgra.ctypes.data if bgra is not None else None,
                                      lin.ctypes.data if lin is not None else None, ctypes.byref(st), dst),
              "rtow_multi_render")
        return bgra, lin, st, list(dst)

    def close(self):
        if self._h:
            lib().rtow_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- tile partition (the host-side statement of decode_pixel / assemble_kernel) ----
def rank_pixels(width, height, rank, world):
    """Framebuffer indices (y*W + x, y from the top) of rank's slab, in slab
    order: slot s holds tile rank + s*world, 64 pixels row-major in the tile.
    Padding pixels of partial tiles are -1."""
    tiles_x = (width + 7) // 8
    n = rank_tile_count(width, height, rank, world)
    slot = np.arange(n, dtype=np.int64)[:, None]
    q = np.arange(64, dtype=np.int64)[None, :]
    tile = rank + slot * world
    x = (tile % tiles_x) * 8 + (q & 7)
    y = (tile // tiles_x) * 8 + (q >> 3)
    idx = np.where((x < width) & (y < height), y * width + x, -1)
    return idx.reshape(-1)


def assemble(slabs, width, height, world):
    """numpy mirror of assemble_kernel: slabs [world, stride_px, C] -> frame [H, W, C]."""
    slabs = np.asarray(slabs)
    frame = np.zeros((height * width,) + slabs.shape[2:], slabs.dtype)
    for r in range(world):
        idx = rank_pixels(width, height, r, world)
        ok = idx >= 0
        frame[idx[ok]] = slabs[r, : idx.size][ok]
    return frame.reshape((height, width) + slabs.shape[2:])
