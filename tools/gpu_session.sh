# round 4 (session 2): the grid walk's height tests without the spatial
# margin (eh) -- A/B against rtw, profile, grid / full-res / fuzz GPU tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SPP=256 AB_ROUNDS=3 AB_SPC=0 AB_SCENES=final_ned timeout -k 10 300 \
    python -u tools/ab.py ab/rtw.so ab/eh.so > gpurun_out/ab_eh.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/prof_counters.py final_ned 32 > gpurun_out/prof_final_ned_eh.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_grid.py tests/test_gpu_fullres.py tests/test_gpu_fuzz.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/gputests_eh.log 2>&1 || exit $?
