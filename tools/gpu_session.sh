# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r03k.log 2>&1 || exit $?
AB_SCENES=final_ned,cornell_smoke AB_SPP=256 AB_ROUNDS=2 timeout -k 10 400 python tools/ab.py ab/lmask.so ab/deadray.so ab/park.so > gpurun_out/ab_park.log 2>&1 || exit $?
timeout -k 10 200 python tools/prof_counters.py final_ned 32 > gpurun_out/prof_final_r03k.log 2>&1 || exit $?
