#!/bin/bash
# Profiles of the bench configuration (run on the GPU box from the repo root):
# rocprofv3 kernel trace + stats, then PMC passes for HBM traffic and the SQ
# breakdown; writes profiles/<TAG>_*.  Usage: bash tools/profile_bench.sh TAG
set -o pipefail
TAG=${1:-r01}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $OUT/trace.log 2>&1 || exit $?
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- \
      python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/p$i.log 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
out, n = {}, {}
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "trace_kernel" in r["Kernel_Name"]:
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
            out["_kernel"] = r["Kernel_Name"][:80]
            out["_vgpr"] = int(r["VGPR_Count"]); out["_lds"] = int(r["LDS_Block_Size"]); out["_grid"] = int(r["Grid_Size"])
json.dump(out, open(sys.argv[1] + "/pmc_summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
