#!/bin/bash
# PMC passes (VALU issue and lane use, wave-cycle split, memory) over the
# trace kernel of each general config's scene (tools/pmc_scene.py), one
# counter group per run.  GPU box, repo root: bash tools/pmc_scenes.sh TAG
set -o pipefail
TAG=${1:-scenes}
R=$(pwd)
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
for sc in "final_ned 1024 1024 64" "cornell_smoke 800 800 64" "cornell 800 800 64" "random_ned 1920 1080 32"; do
  name=$(echo $sc | cut -d' ' -f1)
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32" \
             "SQ_INSTS_VALU_FLOPS_FP64 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $OUT/${name}_p$i -o run --output-format csv -- \
        python3 $R/tools/pmc_scene.py $sc > $OUT/${name}_p$i.log 2>&1 || exit $?
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys, re
out = {}
for d in sorted(glob.glob(sys.argv[1] + "/*_p[0-9]")):
    name = os.path.basename(d).rsplit("_p", 1)[0]
    v = out.setdefault(name, {})
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "trace_kernel" in r["Kernel_Name"]:
                v[r["Counter_Name"]] = v.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
                v["_kernel"] = r["Kernel_Name"][:60]
    m = re.search(r"segments (\d+) kernel_ms ([\d.]+)", open(d + ".log").read())
    v["segments"] = int(m.group(1)); v.setdefault("kernel_ms", []).append(float(m.group(2)))
for name, v in out.items():
    s = v["segments"]
    if "SQ_INSTS_VALU" in v:
        v["valu_per_ray"] = v["SQ_INSTS_VALU"] / s
    if "SQ_THREAD_CYCLES_VALU" in v:
        v["lane_util"] = v["SQ_THREAD_CYCLES_VALU"] / (v["SQ_ACTIVE_INST_VALU"] * 64)
        v["issue_frac"] = v["SQ_ACTIVE_INST_VALU"] / v["SQ_WAVE_CYCLES"]
        v["wait_frac"] = v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"]
        v["dep_stall_frac"] = v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"]
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
for name, v in out.items():
    print(name, {k: (round(x, 4) if isinstance(x, float) else x) for k, x in v.items() if not k.startswith("SQ_") or k in ("SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_FLOPS_FP64")})
PY
