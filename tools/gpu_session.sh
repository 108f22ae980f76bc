# round 4: final_ned's first tree in its own loop (TOP_DTREE) -- A/B against
# the committed build on the general configs, then the GPU suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SPP=256 AB_ROUNDS=3 AB_SPC=0 AB_SCENES=final_ned,cornell,cornell_smoke timeout -k 10 500 \
    python -u tools/ab.py ab/new.so ab/dtree.so ab/dtree.so:RTOW_DTREE=0 > gpurun_out/ab_dtree_r04a.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gputests_dtree_r04a.log 2>&1 || exit $?
