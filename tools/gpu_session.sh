# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/gputests_r03f.log 2>&1
AB_SCENES=cornell_smoke,final_ned,cornell AB_SPP=256 AB_ROUNDS=2 timeout -k 10 300 python tools/ab.py ab/nobvh.so ab/gf.so ab/box.so ab/flags.so > gpurun_out/ab_gf.log 2>&1 || exit $?
AB_SCENES=random_ned AB_SPP=1024 AB_ROUNDS=2 AB_SPC=0 timeout -k 10 300 python tools/ab.py ab/nobvh.so ray-tracing-one-weekend_amd/librtow_hip.so > gpurun_out/ab_rn.log 2>&1 || exit $?
