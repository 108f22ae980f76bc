# round 4 (session 2): grid walk, a row set-up falls through to its first cell
# -- A/B, profile, GPU suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SPP=256 AB_ROUNDS=3 AB_SPC=0 AB_SCENES=final_ned timeout -k 10 300 \
    python -u tools/ab.py ab/grid4.so ab/grid5.so > gpurun_out/ab_grid5.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/prof_counters.py final_ned 32 > gpurun_out/prof_final_ned_grid5.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gputests_grid5.log 2>&1 || exit $?
