# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SCENES=final_ned,cornell_smoke AB_SPP=256 AB_ROUNDS=2 timeout -k 10 400 python tools/ab.py ab/lmask.so ab/scanonly.so ab/treescan.so > gpurun_out/ab_defer.log 2>&1 || exit $?
