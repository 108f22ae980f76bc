"""TEST INFRASTRUCTURE: bench.py's launcher and timed loop on the CPU.

Run as `python tests/bench_stub_worker.py --gpus N ...` without WORLD_SIZE,
bench.main() takes the same path as `python bench.py --gpus N`: it starts N
ranks of this script through a torch.distributed.run child, and every rank
runs bench.run() -- process group, warmup, barrier-bracketed timed steps,
max-over-ranks time, per-rank kernel times, rank 0's JSON line.  The only
difference is the rank object: OracleRank renders its tile slab with the C
oracle (the checker; never part of the product path) on the CPU and talks
gloo, where bench.HipRank renders with librtow_hip.so and talks RCCL.  Rank 0
saves the assembled frame to $RTOW_BENCH_STUB_OUT (tests/test_distributed.py).
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, HERE, os.path.join(REPO, "ray-tracing-one-weekend_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402


class _Stats:
    def __init__(self, cnt, ms):
        self.segments, self.samples, self.kernel_ms = cnt.segments, cnt.samples, ms


class OracleRank:
    backend = "gloo"

    def __init__(self, args, rank, world, local):
        self.args, self.rank, self.world = args, rank, world
        self.device = torch.device("cpu")
        W, H = args.width, args.height
        self.scene = bench.build_scene(args)
        self.cam = sio.RtowCamera.from_buffer_copy(bytes(rtow.camera_main(W, H)))
        self.p = sio.default_params(W, H, args.spp, seed=args.seed)
        self.idx = rtow.rank_pixels(W, H, rank, world)
        self.valid = self.idx >= 0
        self.stride = rtow.rank_tile_count(W, H, 0, world) * 64
        self.slab = torch.zeros(self.stride * 4, dtype=torch.uint8)
        self.gathered = torch.zeros((world, self.stride * 4), dtype=torch.uint8) if rank == 0 else None
        self.frame = None

    def init_kwargs(self):
        return {}

    def _render(self, sl):
        t0 = time.perf_counter()
        _, bgra, cnt = sio.oracle_render(self.scene.view_ptr, self.cam, self.p,
                                         pixels=self.idx[self.valid].astype(np.uint32), threads=2)
        view = sl.view(self.stride, 4)
        view[: self.idx.size][torch.from_numpy(self.valid)] = torch.from_numpy(bgra.reshape(-1, 4))
        return _Stats(cnt, (time.perf_counter() - t0) * 1e3)

    def _assemble(self, g):
        self.frame = rtow.assemble(g.view(self.world, self.stride, 4).numpy(), self.args.width, self.args.height,
                                   self.world)

    def step(self, dist):
        return bench.frame_step(self._render, self._assemble, self.slab, self.gathered, self.rank, self.world, dist)

    def sync(self):
        pass

    def report(self, segs, steps, mean_kms):
        return {"stub": "C oracle render on the CPU (tests/bench_stub_worker.py), gloo"}

    def close(self):
        if self.rank == 0 and os.environ.get("RTOW_BENCH_STUB_OUT"):
            np.save(os.environ["RTOW_BENCH_STUB_OUT"], self.frame)


if __name__ == "__main__":
    bench.main(make_rank=OracleRank)
