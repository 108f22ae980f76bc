#!/bin/bash
# Profile recipe for round 1 (run on the GPU box from the repo root):
# bench line, rocprofv3 kernel trace + stats, then PMC passes (one counter
# group per pass, --kernel-trace only beside them).
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $OUT/prof_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/prof_fetch -o run --output-format csv -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/prof_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/prof_write -o run --output-format csv -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/prof_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/prof_sq -o run --output-format csv -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/prof_sq.log 2>&1 || exit $?
echo done
