# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/gputests_r03e.log 2>&1
AB_SCENES=cornell_smoke,final_ned,cornell AB_SPP=256 AB_ROUNDS=2 timeout -k 10 300 python tools/ab.py ab/nobvh.so ab/tie.so > gpurun_out/ab_tie.log 2>&1 || exit $?
timeout -k 10 120 python tools/tie_measure.py > gpurun_out/tie_measure_e.log 2>&1 || exit $?
timeout -k 10 200 python tools/prof_counters.py random_ned 64 > gpurun_out/prof_random_r03e.log 2>&1 || exit $?
