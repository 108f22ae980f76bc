# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SCENES=final_ned AB_SPP=256 AB_ROUNDS=2 timeout -k 10 400 python tools/ab.py ab/park.so ab/defer.so:RTOW_BOX_DEFER=1 ab/defer.so:RTOW_BOX_DEFER=8 ab/defer.so:RTOW_BOX_DEFER=16 ab/defer.so:RTOW_BOX_DEFER=32 ab/defer.so:RTOW_BOX_DEFER=48 > gpurun_out/ab_defer2.log 2>&1 || exit $?
RTOW_BOX_DEFER=16 timeout -k 10 200 python tools/prof_counters.py final_ned 32 > gpurun_out/prof_final_r03m.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r03l.log 2>&1 || exit $?
