"""Summarise the PMC passes of tools/profile_bench.sh into pmc_summary.json.

For every pass directory OUT/p*/ the trace kernel's counters (one launch: the
passes run bench.py --steps 1 --warmup 0) are read from rocprofv3's
counter-collection CSV; the pass's bench line (OUT/p*.log) gives the rays that
launch traced and its kernel time.  The summary records the build's source
hash (rtow.source_hash()) and the bench config, so bench.py uses it only for
the build and config it describes.

  python3 tools/pmc_summarize.py gpurun_out/prof_TAG
"""
import csv
import glob
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "ray-tracing-one-weekend_amd"))
import rtow  # noqa: E402


def bench_line(log):
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise SystemExit(f"no bench line in {log}")


def main(out):
    summary = {"source_hash": rtow.source_hash(), "created": int(time.time())}
    passes = {}
    for d in sorted(glob.glob(os.path.join(out, "p[0-9]*"))):
        if not os.path.isdir(d):
            continue
        name = os.path.basename(d)
        b = bench_line(d + ".log")
        cfg = b["config"]
        config = [cfg["width"], cfg["height"], cfg["spp"], cfg["n"], b["n_gpus"]]
        summary.setdefault("workload", cfg.get("scene", "random_ned"))
        if summary.setdefault("config", config) != config:
            raise SystemExit(f"{name}: config {config} differs from {summary['config']}")
        rays = b["rays_per_step"]
        kms = b["roofline"]["kernel_ms"]
        # per dispatch (bench.py's rank setup renders one 1-spp frame before
        # the step: the step's launch is the trace_kernel dispatch with the
        # largest counter values)
        disp, kernel = {}, None
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "trace_kernel" not in r["Kernel_Name"]:
                    continue
                v = disp.setdefault(r.get("Dispatch_Id") or r.get("Correlation_Id"), {})
                v[r["Counter_Name"]] = v.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                kernel = r["Kernel_Name"][:96]
                summary["_vgpr"] = int(r.get("VGPR_Count") or r.get("Arch_VGPR_Count") or 0)
                summary["_grid"] = int(r["Grid_Size"])
        if not disp:
            raise SystemExit(f"{name}: no trace_kernel counters")
        vals = max(disp.values(), key=lambda v: sum(v.values()))
        # counters per launch, normalised to the first pass's ray count (the
        # launches trace the same frame; ray counts agree to the last ray)
        rays0 = summary.setdefault("rays_per_launch", rays)
        for k, v in vals.items():
            summary[k] = v * rays0 / rays
        passes[name] = {"rays": rays, "kernel_ms": kms, "counters": sorted(vals)}
        if "GRBM_GUI_ACTIVE" in vals:
            summary["kernel_ms_pmc"] = kms
        summary["_kernel"] = kernel
    summary["passes"] = passes
    if "SQ_INSTS_VALU" in summary:
        summary["valu_per_ray"] = summary["SQ_INSTS_VALU"] / summary["rays_per_launch"]
    if "SQ_THREAD_CYCLES_VALU" in summary:
        summary["lane_util"] = summary["SQ_THREAD_CYCLES_VALU"] / (summary["SQ_ACTIVE_INST_VALU"] * 64)
    json.dump(summary, open(os.path.join(out, "pmc_summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
