#!/bin/bash
# Profiles of the bench configuration (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats of bench.py (per-kernel durations;
#      3 steps, no prime launch: every trace-kernel call is a bench step),
#   2. PMC passes, one counter group per run with --kernel-trace beside it
#      only (never a trace domain), each over ONE bench step (one launch),
# then tools/pmc_summarize.py writes pmc_summary.json: the trace kernel's
# counters per launch, tagged with the build's source hash, the config and
# the rays of that launch -- what bench.py's VALU roofline reads; and last
#   3. bench.py itself (the line the driver parses, CPU baseline included),
#      its roofline from that summary.
#   bash tools/profile_bench.sh TAG [extra bench.py args, e.g. --workload cornell]
# Output: gpurun_out/prof_TAG/ (copy bench.json, kernel_stats.csv and
# pmc_summary.json into profiles/TAG/).
set -o pipefail
TAG=${1:-r02}
shift
EXTRA="$*"
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 0 --no-prime --no-cpu $EXTRA > $OUT/trace.log 2>&1 || exit $?
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- \
      python3 $R/bench.py --steps 1 --warmup 0 --no-cpu $EXTRA > $OUT/p$i.log 2>&1 || exit $?
done
cd $R
python3 tools/pmc_summarize.py $OUT || exit $?
# the bench line last, its roofline from the counters just summarized
timeout -k 10 300 python3 bench.py $EXTRA --pmc-json $OUT/pmc_summary.json > $OUT/bench.json 2> $OUT/bench.err || exit $?
