#!/usr/bin/env python3
"""Benchmark of the per-pixel render loop (main.cpp:932-996) on N MI355X.

Default workload: BASELINE.json config 2 -- the book-1 random scene
(randomScene_NED with n = 487, 488 hitables under one BvhNode) at
1920x1080x1024spp, depth 50.  `--workload final_ned` is config 5 (book-2
final_scene, 4096x4096x8192spp, quoted for 8 GPUs); cornell / cornell_smoke
are configs 3 / 4.

One step = one full frame: every rank renders its share of the frame's 8x8
tiles (rank r takes tiles r, r+N, ...; the reference's column interleave,
main.cpp:936, at tile granularity) with the HIP path in librtow_hip.so, then
one RCCL gather (torch.distributed, backend "nccl") brings the tile slabs to
rank 0, which assembles the BGRA frame on its GPU.  Total work is the fixed
frame, so scaling is "strong".

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--spp S] [--no-cpu]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

`--gpus N > 1` without a torch.distributed environment (WORLD_SIZE unset)
starts N ranks itself (a torch.distributed.run child, before this process
touches a GPU) and exits with its status; a WORLD_SIZE that differs from
--gpus is an error.  A multi-GPU request never silently runs one rank.

Rank 0 prints ONE JSON line (value = whole-job Mray/s; Msample/s beside it;
`rank_kernel_ms` the trace kernel's time on every rank).

roofline: the bound that limits this kernel is VALU issue, not HBM (the scene
is LDS/L2-resident; measured HBM traffic is ~7 GB/s).  achieved = VALU
wave-instructions per second of the trace kernel = (wave-instructions per ray,
SQ_INSTS_VALU from the committed rocprofv3 PMC pass of this exact build and
workload, profiles/<round>_*/pmc_summary.json) x the rays this launch traced /
the kernel's mean duration from HIP events on the render stream.  peak = 1024
SIMDs x 2.4 GHz x 0.5 (a wave64 VALU instruction occupies a SIMD-32 for two
cycles, MI355X_MICROARCH.md).  lane_util = the active-lane fraction of those
instructions (SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64), calibrated on
gfx950 by tools/valu_calib.hip), so frac x lane_util is the useful-lane share
of the chip's VALU throughput.  The measured HBM bytes (FETCH_SIZE x 2 +
WRITE_SIZE of the same PMC run) and the reference-equivalent record bytes per
ray are informational fields.  cpu_baseline = the reference's
own code (oracle/_ref/ref_harness) on all the host cores this process may use
over a bounded random pixel sample, rays counted by the C oracle on the same
pixels (the oracle alone, kind "port", when the harness was not built);
`as_written` beside it times the reference with its own shared, racy
std::mt19937_64 (rngs.h:9-11).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-one-weekend_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMD-32, a wave64 VALU instruction takes two
# cycles of its SIMD, 2.4 GHz max clock (MI355X_MICROARCH.md) -> G wave-instr/s
N_SIMD, CLOCK_GHZ = 1024, 2.4
VALU_PEAK_G = N_SIMD * CLOCK_GHZ * 0.5
# algorithmic record bytes per reference traversal event
BYTES_BVH, BYTES_SPHERE, BYTES_MSPHERE, BYTES_RECT, BYTES_MEDIUM = 32, 20, 40, 24, 8

# BASELINE.json configs by name: scene, n, W, H, spp, the world the config is quoted for, label
WORKLOADS = {
    "random_ned": ("random_ned", 487, 1920, 1080, 1024, "book-1 random_scene"),
    "cornell": ("cornell", 0, 800, 800, 4096, "cornell_box"),
    "cornell_smoke": ("cornell_smoke", 0, 800, 800, 4096, "cornell_smoke"),
    "final_ned": ("final_ned", 0, 4096, 4096, 8192, "book-2 final_scene"),
}
BASELINE_METRIC = "Mray/s + Msample/s, random_scene 1920×1080×1024spp at 1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="random_ned")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--texture", choices=["earth", "synthetic"], default="earth",
                    help="earth: the reference's input_images/1_earth_8k.jpg (scenes.h:140), staged in the repo; "
                         "synthetic: rtow_synthetic_image's 2048x1024 stand-in")
    ap.add_argument("--cpu-pixels", type=int, default=None,
                    help="pixels of the CPU baseline's sample (default: ~10-20 s of the reference's work)")
    ap.add_argument("--cpu-spp", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-prime", action="store_true",
                    help="skip the 1-spp render that loads the code objects (profiling: every trace-kernel launch is a step)")
    ap.add_argument("--cpu-kind", choices=["auto", "port"], default="auto",
                    help="auto: the reference's own code when oracle/_ref was built, else the oracle")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every host CPU this process may use")
    ap.add_argument("--inproc", action="store_true",
                    help="one process drives all --gpus N devices through the C-ABI's own multi-GPU render "
                         "(rtow_multi_render: a host thread per device, one RCCL gather, assembly on device 0; "
                         "every rank chunks as the whole frame), instead of one process per GPU")
    ap.add_argument("--share-device", action="store_true",
                    help="(test mode, not a bench line) every rank renders on cuda:0 and the slabs are gathered "
                         "with gloo through host memory: the multi-process path with real kernels on a one-GPU box")
    ap.add_argument("--frame-plan", action="store_true",
                    help="every rank chunks its samples as the whole frame (RTOW_FLAG_FRAME_PLAN): the assembled "
                         "frame equals a one-GPU rtow_render bit for bit")
    ap.add_argument("--dump-frame", default=None,
                    help="rank 0 writes the last step's assembled BGRA frame (H x W x 4 bytes) to this file")
    ap.add_argument("--pmc-json", default=None,
                    help="PMC summary to use (default: the newest profiles/*/pmc_summary.json of this build+config)")
    args = ap.parse_args(argv)
    scene, n, W, H, spp, _ = WORKLOADS[args.workload]
    args.scene = scene
    args.n = n if args.n is None else args.n
    args.width = W if args.width is None else args.width
    args.height = H if args.height is None else args.height
    args.spp = spp if args.spp is None else args.spp
    if args.cpu_spp is None:
        args.cpu_spp = min(args.spp, 1024)
    if args.cpu_pixels is None:  # ~10-20 s of the reference's code on 16 host cores
        args.cpu_pixels = {"random_ned": 40000, "cornell": 8000, "cornell_smoke": 8000, "final_ned": 3000}[args.workload]
    return args


# ---------------------------------------------------------------------------
# launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(nproc, argv, script=None):
    """Start `nproc` ranks of `script` (default: this file) with argv through a
    torch.distributed.run child on 127.0.0.1 and return its exit status.  The
    caller must not have touched a GPU (the child, not an exec, runs them)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(script or __file__)] + list(argv)
    return subprocess.run(cmd).returncode


EARTH = os.path.join(REPO, "input_images", "1_earth_8k.jpg")


def build_scene(args):
    """The benched world: the reference's scene builder restated
    (rtow_build_scene), with the reference's own earth texture
    (input_images/1_earth_8k.jpg, loaded as scenes.h:140 does) unless
    --texture synthetic."""
    import rtow

    if args.texture == "earth":
        if not os.path.exists(EARTH):
            raise SystemExit(f"bench: {EARTH} is missing (--texture synthetic renders without it)")
        return rtow.Scene.build(args.scene, n=max(args.n, 1), image="jpeg", image_path=EARTH, scene_seed=1)
    return rtow.Scene.build(args.scene, n=max(args.n, 1), image="synthetic", scene_seed=1)


# ---------------------------------------------------------------------------
# CPU baseline
def reference_run(pix, args, threads, racy=False):
    """The reference's own code (oracle/_ref/ref_harness, compiled from
    /root/reference's headers in the build container; its render loop body is
    main.cpp:938-951) on the same pixels: (seconds, checksum) or None when the
    harness was not built.  racy: with the reference's own shared
    std::mt19937_64 (rngs.h:9-11) instead of the seeded counter engine.  The
    scenes load their earth texture from ./input_images/1_earth_8k.jpg
    (scenes.h:140): the repo's copy of that file, or with --texture synthetic
    the synthetic texture staged there as a lossless PNG."""
    import shutil
    import tempfile

    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if not os.access(harness, os.X_OK):
        return None
    try:
        from PIL import Image

        import rtow
    except ImportError:
        return None
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "input_images"))
        if args.texture == "earth":
            shutil.copy(EARTH, os.path.join(d, "input_images", "1_earth_8k.jpg"))
        else:
            Image.fromarray(rtow.synthetic_image(2048, 1024), "RGB").save(
                os.path.join(d, "input_images", "1_earth_8k.jpg"), format="PNG")
        pf = os.path.join(d, "pix.u32")
        pix.tofile(pf)
        env = dict(os.environ, RTOW_SCENE_SEED="1")
        cmd = [harness, "bench", args.scene, str(args.width), str(args.height), str(args.cpu_spp), pf,
               "--n", str(max(args.n, 1)), "--seed", str(args.seed), "--threads", str(threads), "--cwd", d]
        out = subprocess.run(cmd + (["--racy"] if racy else []), env=env, capture_output=True, text=True,
                             timeout=600)
    if out.returncode != 0:
        return None
    r = json.loads(out.stdout.strip().splitlines()[-1])
    return r["seconds"], r["checksum"]


def cpu_baseline(scene, cam, args, threads):
    """The CPU render of a bounded random pixel sample of the same frame: the
    reference's own code (kind "reference", oracle/_ref) when it was built, the
    oracle otherwise (kind "port": the reference's render loop restated in C,
    bit-exact with the reference build).  The oracle always runs: its traversal
    counts give the ray count (the same paths: the two agree bit for bit, and
    the checksum of the pixel sums shows it) and bytes/ray."""
    import scene_io as sio

    rng = np.random.default_rng(1234)
    W, H = args.width, args.height
    pix = rng.choice(W * H, size=min(args.cpu_pixels, W * H), replace=False).astype(np.uint32)
    ocam = sio.RtowCamera.from_buffer_copy(bytes(cam))
    p = sio.default_params(W, H, args.cpu_spp, seed=args.seed)
    t0 = time.perf_counter()
    lin, _, c = sio.oracle_render(scene.view_ptr, ocam, p, pixels=pix, threads=threads)
    dt = time.perf_counter() - t0
    bytes_per_ray = (c.bvh_visits * BYTES_BVH + c.sphere_tests * BYTES_SPHERE + c.moving_sphere_tests * BYTES_MSPHERE
                     + c.rect_tests * BYTES_RECT + c.medium_calls * BYTES_MEDIUM) / max(c.segments, 1)
    sample = f"{len(pix)} random pixels of the {W}x{H} frame x {args.cpu_spp} spp (same scene/seed), {threads} threads"
    port = {"value": round(c.segments / dt / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
            "msample_per_s": round(c.samples / dt / 1e6, 4), "seconds": round(dt, 2),
            "sample": sample + ", oracle/librtow_oracle.so"}
    base = port
    print(f"cpu_baseline: oracle {dt:.1f} s; the reference's own code next", file=sys.stderr, flush=True)
    ref = reference_run(pix, args, threads) if args.cpu_kind != "port" else None
    if ref is not None:
        rs, checksum = ref
        osum = float(lin.astype(np.float64).sum())
        base = {"value": round(c.segments / rs / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": "reference",
                "msample_per_s": round(c.samples / rs / 1e6, 4), "seconds": round(rs, 2),
                "sample": sample + ", oracle/_ref/ref_harness (the reference's headers); rays counted by the oracle",
                "same_result_as_oracle": bool(abs(checksum - osum) <= 1e-6 * max(1.0, abs(osum))),
                "port": {k: port[k] for k in ("value", "msample_per_s", "seconds")}}
        print(f"cpu_baseline: reference {rs:.1f} s; the reference as written next", file=sys.stderr, flush=True)
        racy = reference_run(pix, args, threads, racy=True)
        if racy is not None:
            # its paths differ from the seeded ones (other random numbers):
            # rays estimated from the oracle's rays per sample on the same pixels
            base["as_written"] = {
                "value": round(c.segments / racy[0] / 1e6, 3), "unit": "Mray/s",
                "msample_per_s": round(c.samples / racy[0] / 1e6, 4), "seconds": round(racy[0], 2),
                "note": "the reference as written: every thread draws from the one shared std::mt19937_64 "
                        "(rngs.h:9-11, main.cpp:942-943) unsynchronised -- a data race, so not reproducible; "
                        "rays = samples x the seeded run's rays per sample"}
    counts = {"segments_per_sample": c.segments / max(c.samples, 1),
              "bvh_visits_per_ray": c.bvh_visits / max(c.segments, 1),
              "sphere_tests_per_ray": c.sphere_tests / max(c.segments, 1),
              "moving_sphere_tests_per_ray": c.moving_sphere_tests / max(c.segments, 1)}
    return base, bytes_per_ray, counts


# ---------------------------------------------------------------------------
# roofline
def pmc_key(args, world):
    """What a PMC summary must describe to price this run."""
    return {"workload": args.scene, "config": [args.width, args.height, args.spp, args.n, world]}


def find_pmc(args, world, src_hash):
    """The PMC summary (tools/profile_bench.sh) that describes this run: the
    newest one under profiles/ recorded for this workload, config and build
    source hash; failing that the newest for this workload and config, flagged
    stale.  "Newest" is the summary's own `created` stamp (unix seconds, from
    tools/pmc_summarize.py), then the file's mtime."""
    import glob

    cands = [args.pmc_json] if args.pmc_json else glob.glob(os.path.join(REPO, "profiles", "*", "pmc_summary.json"))
    want = pmc_key(args, world)
    fresh, stale = [], []
    for f in cands:
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload", "random_ned") != want["workload"] or d.get("config") != want["config"]:
            continue
        if "SQ_INSTS_VALU" not in d:
            continue
        age = (d.get("created", 0), os.path.getmtime(f))
        (fresh if d.get("source_hash") == src_hash else stale).append((age, f, d))
    for group in (fresh, stale):
        if group:
            _, f, d = max(group, key=lambda e: e[0])
            return f, d
    return None


def roofline(args, world, launch_rays, mean_kms, bpr, src_hash):
    """VALU-issue roofline of the trace kernel (see the module docstring)."""
    found = find_pmc(args, world, src_hash)
    if found is None:
        return {"bound": "valu", "achieved": None, "peak": VALU_PEAK_G, "unit": "Gwave-instr/s", "frac": None,
                "traffic": None, "kernel_ms": round(mean_kms, 2), "note": "no PMC summary for this config under profiles/"}
    path, d = found
    rays_pmc = d["rays_per_launch"]
    valu_per_ray = d["SQ_INSTS_VALU"] / rays_pmc
    achieved = valu_per_ray * launch_rays / (mean_kms * 1e-3) / 1e9
    lane_util = d["SQ_THREAD_CYCLES_VALU"] / (d["SQ_ACTIVE_INST_VALU"] * 64) if "SQ_THREAD_CYCLES_VALU" in d else None
    traffic = None
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:  # KB; FETCH_SIZE reads half the bytes on gfx950
        traffic = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024 / rays_pmc * launch_rays
    frac = achieved / VALU_PEAK_G
    roof = {"bound": "valu", "achieved": round(achieved, 1), "peak": VALU_PEAK_G, "unit": "Gwave-instr/s",
            "frac": round(frac, 4),
            "lane_util": round(lane_util, 4) if lane_util is not None else None,
            "useful_lane_frac": round(frac * lane_util, 4) if lane_util is not None else None,
            "traffic": round(traffic) if traffic is not None else None,
            "valu_per_ray": round(valu_per_ray, 3), "kernel_ms": round(mean_kms, 2),
            "pmc": os.path.relpath(path, REPO), "pmc_source_hash": d.get("source_hash"),
            "pmc_matches_build": d.get("source_hash") == src_hash,
            "peak_def": f"{N_SIMD} SIMD-32 x {CLOCK_GHZ} GHz x 0.5 wave64 VALU instr/cycle"}
    if "WRITE_SIZE" in d:
        roof["write_bytes"] = round(d["WRITE_SIZE"] * 1024 / rays_pmc * launch_rays)
    if "GRBM_GUI_ACTIVE" in d and d.get("kernel_ms_pmc"):
        roof["clock_ghz_under_pmc"] = round(d["GRBM_GUI_ACTIVE"] / 8 / (d["kernel_ms_pmc"] * 1e-3) / 1e9, 3)
    if traffic is not None:
        roof["hbm_gbps"] = round(traffic / (mean_kms * 1e-3) / 1e9, 2)
        roof["hbm_frac"] = round(traffic / (mean_kms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5)
    if bpr is not None:
        roof["reference_bytes_per_ray"] = round(bpr, 1)
        roof["reference_equiv_gbps"] = round(bpr * launch_rays / (mean_kms * 1e-3) / 1e9, 1)
    roof["bound_note"] = ("VALU issue bounds this kernel, not HBM: the scene is LDS/L2-resident (hbm_frac is the "
                          "measured DRAM traffic over 8 TB/s); reference_equiv_gbps prices the record bytes the "
                          "reference's exhaustive traversal reads (SURVEY 8d), which the SAH traversal never "
                          "fetches -- informational, not a hardware bound (DESIGN.md 'Roofline and measurement')")
    return roof


# ---------------------------------------------------------------------------
# one step
def frame_step(render, assemble, slab, gathered, rank, world, dist=None, host_gather=False):
    """One bench step: this rank renders its 8x8-tile slab (`render(slab)`),
    one gather brings every rank's slab to rank 0 (torch.distributed: RCCL
    over xGMI on the GPUs, gloo in tests/test_distributed.py), rank 0
    assembles the frame (`assemble(gathered)`).  host_gather: the slabs go
    through host memory (gloo between processes sharing one GPU,
    --share-device).  Returns render's stats."""
    st = render(slab)
    if world > 1 and host_gather:
        hs = slab.cpu()
        hg = [h.clone() for h in gathered.cpu().unbind(0)] if rank == 0 else None
        dist.gather(hs, hg, dst=0)
        if rank == 0:
            for r in range(world):
                gathered[r].copy_(hg[r])
    elif world > 1:
        dist.gather(slab, list(gathered.unbind(0)) if rank == 0 else None, dst=0)
    else:
        gathered[0].copy_(slab)
    if rank == 0:
        assemble(gathered)
    return st


class HipRank:
    """One rank of the product path: librtow_hip.so on cuda:LOCAL_RANK, RCCL
    (torch.distributed backend "nccl") between ranks."""

    backend = "nccl"

    def __init__(self, args, rank, world, local):
        import torch

        import rtow

        self.args, self.rank, self.world = args, rank, world
        if args.share_device:  # (test mode) every rank on the one GPU, gloo between them
            local = 0
            self.backend = "gloo"
        torch.cuda.set_device(local)
        self.device = torch.device("cuda", local)
        W, H = args.width, args.height
        self.scene = build_scene(args)
        self.cam = rtow.camera_main(W, H)
        self.ctx = rtow.Context(local)
        self.ctx.upload(self.scene)
        self.stride = rtow.rank_tile_count(W, H, 0, world) * 64  # rank 0 holds the most tiles
        self.slab = torch.zeros(self.stride * 4, dtype=torch.uint8, device=self.device)
        self.gathered = torch.zeros((world, self.stride * 4), dtype=torch.uint8, device=self.device) if rank == 0 else None
        self.frame = torch.zeros((H, W, 4), dtype=torch.uint8, device=self.device) if rank == 0 else None
        self.stream = torch.cuda.current_stream().cuda_stream
        self.p = rtow.params(W, H, args.spp, seed=args.seed, rank=rank, world=world,
                             flags=rtow.FLAG_FRAME_PLAN if args.frame_plan else 0)
        # load the code objects once (not a step: the warmup steps stay the contract's)
        if not args.no_prime:
            self.ctx.render_tiles_device(self.cam, rtow.params(W, H, 1, seed=args.seed, rank=rank, world=world),
                                         self.slab.data_ptr(), None, self.stream)
        torch.cuda.synchronize()

    def init_kwargs(self):
        return {} if self.args.share_device else {"device_id": self.device}

    def step(self, dist):
        W, H = self.args.width, self.args.height
        return frame_step(
            lambda sl: self.ctx.render_tiles_device(self.cam, self.p, sl.data_ptr(), None, self.stream),
            lambda g: self.ctx.assemble_device(W, H, self.world, g.data_ptr(), self.stride, self.frame.data_ptr(),
                                               self.stream),
            self.slab, self.gathered, self.rank, self.world, dist, host_gather=self.args.share_device)

    def dump_frame(self, path):
        if self.rank == 0:
            self.frame.cpu().numpy().tofile(path)

    def sync(self):
        import torch

        torch.cuda.synchronize()

    def report(self, segs, steps, mean_kms):
        """Rank 0's extra fields: cpu_baseline (N=1 only) and the roofline."""
        import rtow

        args, world = self.args, self.world
        threads, cpu_info = rtow.host_threads()
        if args.cpu_threads:
            threads = args.cpu_threads
        if args.no_cpu:
            base, bpr, counts = None, None, {}
        elif world == 1:
            base, bpr, counts = cpu_baseline(self.scene, self.cam, args, threads)
            base.update(cpu_info)
        else:  # the CPU baseline is quoted at N=1 only; bytes/ray from a smaller oracle sample
            args.cpu_pixels = max(1, args.cpu_pixels // 10)
            args.cpu_kind = "port"
            _, bpr, counts = cpu_baseline(self.scene, self.cam, args, threads)
            base = None
        launch_rays = segs / max(steps, 1)
        return {"roofline": roofline(args, world, launch_rays, mean_kms, bpr, rtow.source_hash()),
                "cpu_baseline": base,
                "oracle_counts": {k: round(v, 3) for k, v in counts.items()}}

    def close(self):
        self.ctx.close()


class InprocRank(HipRank):
    """--inproc: the C-ABI's multi-GPU render in this one process --
    rtow_multi_render over devices 0..N-1 (rtow_multi.cpp: one rtow_context and
    stream per device, all rendering at once from their own host threads, one
    RCCL gather of the tile slabs to device 0, the BGRA frame assembled there
    and left on the device, as the default path leaves it).  What main.cpp's
    binding would call; no torch.distributed."""

    backend = None

    def __init__(self, args, rank, world, local):
        import torch

        import rtow

        assert world == 1 and rank == 0, "--inproc runs as one process"
        self.args, self.rank = args, 0
        self.world = self.n_gpus = args.gpus
        torch.cuda.set_device(0)
        self.device = torch.device("cuda", 0)
        W, H = args.width, args.height
        self.scene = build_scene(args)
        self.cam = rtow.camera_main(W, H)
        self.multi = rtow.Multi(list(range(self.n_gpus)))
        self.multi.upload(self.scene)
        self.p = rtow.params(W, H, args.spp, seed=args.seed)
        self.device_kms = []
        if not args.no_prime:
            self.multi.render(self.cam, rtow.params(W, H, 1, seed=args.seed), linear=False, host=False)

    def step(self, dist):
        _, _, st, dst = self.multi.render(self.cam, self.p, linear=False, host=False)
        self.device_kms.append([d.kernel_ms for d in dst])
        return st

    def report(self, segs, steps, mean_kms):
        # the roofline prices one device's kernel: its share of the rays (the
        # 8x8-tile interleave balances the shares within ~0.5 %) over the
        # slowest device's kernel time
        return super().report(segs / self.n_gpus, steps, mean_kms)

    def close(self):
        self.multi.close()


def run(args, make_rank):
    """The timed loop of every rank: W warmup steps, then exactly K steps
    between barrier + device synchronize on both sides; the whole-job rate is
    all ranks' rays over the slowest rank's time.  Rank 0 prints the line.

    Only that line goes to stdout: the process's fd 1 points at stderr while
    the run lasts (RCCL prints its version banner to stdout when it creates a
    communicator), and the line is written to the original stdout."""
    sys.stdout.flush()
    line_fd = os.dup(1)
    os.dup2(2, 1)
    try:
        _run(args, make_rank, line_fd)
    finally:
        sys.stdout.flush()
        os.dup2(line_fd, 1)
        os.close(line_fd)


def _run(args, make_rank, line_fd):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    R = make_rank(args, rank, world, local)
    distributed = world > 1
    n_gpus = getattr(R, "n_gpus", world)  # --inproc: one process, N devices
    if args.share_device:  # (test mode) every rank process on the one GPU
        n_gpus = 1
    if distributed:
        dist.init_process_group(R.backend, **R.init_kwargs())

    def barrier():
        if distributed:
            dist.barrier()

    for _ in range(args.warmup):
        R.step(dist)
    barrier()
    R.sync()
    t0 = time.perf_counter()
    segs, samples, kms = 0, 0, []
    for _ in range(args.steps):
        st = R.step(dist)
        segs += st.segments
        samples += st.samples
        kms.append(st.kernel_ms)
    R.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    if getattr(args, "dump_frame", None) and hasattr(R, "dump_frame"):
        R.dump_frame(args.dump_frame)
    mean_kms = float(np.mean(kms)) if kms else 0.0
    cdev = torch.device("cpu") if R.backend == "gloo" else R.device  # (gloo collectives on host tensors)
    tot = torch.tensor([float(segs), float(samples)], dtype=torch.float64, device=cdev)
    el = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    rk = torch.tensor([mean_kms], dtype=torch.float64, device=cdev)
    rank_kms = [rk.clone() for _ in range(world)]
    if distributed:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_gather(rank_kms, rk)
    segs_all, samples_all, elapsed = float(tot[0]), float(tot[1]), float(el[0])
    per_rank = [round(float(t[0]), 2) for t in rank_kms]
    if getattr(R, "device_kms", None):  # --inproc: every device's mean kernel time
        per_rank = [round(float(x), 2) for x in np.mean(np.asarray(R.device_kms), axis=0)]

    if rank == 0:
        scene, _, W0, H0, spp0, label = WORKLOADS[args.workload]
        W, H, spp = args.width, args.height, args.spp
        is_baseline_cfg = args.workload == "random_ned" and (W, H, spp, args.n) == (W0, H0, spp0, 487)
        # the metric names the frame this run rendered (the BASELINE metric only for config 2 exactly)
        metric = BASELINE_METRIC if is_baseline_cfg else f"Mray/s + Msample/s, {label} {W}×{H}×{spp}spp"
        out = {
            "metric": metric,
            "value": round(segs_all / elapsed / 1e6, 2),
            "unit": "Mray/s",
            "msample_per_s": round(samples_all / elapsed / 1e6, 3),
            "n_gpus": n_gpus,
            "ranks": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / max(args.steps, 1), 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("the reference's scene (seeded builder) and its own earth texture input_images/1_earth_8k.jpg"
                     if args.texture == "earth" else "synthetic"),
            "config": {"workload": (f"randomScene_NED n={args.n} ({args.n + 1} hitables under one BvhNode), "
                                    if scene == "random_ned" else f"{label} ({scene}), ")
                                   + f"{W}x{H}x{spp}spp, depth 50, "
                                   + ("earth texture input_images/1_earth_8k.jpg (2048x1024 JPEG)" if args.texture == "earth"
                                      else "synthetic 2048x1024 earth texture"),
                       "scene": scene, "width": W, "height": H, "spp": spp, "n": args.n, "scene_seed": 1,
                       "render_seed": args.seed, "baseline_config": is_baseline_cfg and not args.share_device,
                       "parallelism": (f"tiles8x8 interleaved over {n_gpus} device(s) of one process "
                                       "(rtow_multi_render: RCCL gather to device 0)" if args.inproc else
                                       f"tiles8x8 interleaved over {world} rank processes sharing cuda:0 + gloo "
                                       "gather through host memory (test mode, not a multi-GPU measurement)"
                                       if args.share_device else
                                       f"tiles8x8 interleaved over {world} rank(s) + gather to rank 0")},
            "rays_per_sample": round(segs_all / max(samples_all, 1), 4),
            "rays_per_step": int(segs_all / max(args.steps, 1)),
            "rank_kernel_ms": {"min": min(per_rank), "max": max(per_rank), "per_rank": per_rank},
        }
        out.update(R.report(segs, args.steps, mean_kms))
        os.write(line_fd, (json.dumps(out) + "\n").encode())
    R.close()
    if distributed:
        dist.destroy_process_group()


def main(make_rank=HipRank, argv=None):
    args = parse(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if args.inproc:
        if world_env not in (None, "1"):
            print("bench.py: --inproc is one process; do not launch it with torch.distributed", file=sys.stderr)
            sys.exit(2)
        run(args, InprocRank if make_rank is HipRank else make_rank)
        return
    if world_env is None and args.gpus > 1:
        # N ranks were asked for and none were launched: start them (one
        # process per GPU) instead of running one rank and reporting it
        sys.exit(launch(args.gpus, sys.argv[1:] if argv is None else argv, script=sys.argv[0]))
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    run(args, make_rank)


if __name__ == "__main__":
    main()
