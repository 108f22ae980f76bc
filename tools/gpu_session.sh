# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r03w.log 2>&1
rc=$?
# test failures (1) still allow the A/B; a hang, a kill or a crash ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AB_SCENES=random_ned,final_ned AB_SPP=256 AB_ROUNDS=5 timeout -k 10 600 python -u tools/ab.py ab/v7.so ab/v8.so > gpurun_out/ab_v8.log 2>&1 || exit $?
exit $rc
