# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r03o.log 2>&1 || exit $?
AB_SCENES=final_ned,cornell_smoke,cornell AB_SPP=256 AB_ROUNDS=3 timeout -k 10 500 python tools/ab.py ab/medfast.so ab/chainx.so > gpurun_out/ab_chainx.log 2>&1 || exit $?
