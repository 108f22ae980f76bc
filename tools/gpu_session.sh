# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SCENES=final_ned,cornell_smoke AB_SPP=256 AB_ROUNDS=2 timeout -k 10 300 python tools/ab.py ab/nobvh.so ab/box.so ab/lmask.so > gpurun_out/ab_lmask.log 2>&1 || exit $?
bash tools/round_check.sh r03 > gpurun_out/round_check_r03.log 2>&1
