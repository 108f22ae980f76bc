# round 4 (session 2): the ground's rest as a tree (RTOW_RUNTREE=3) and the
# grid walk with per-ray absolute widenings (rtw) -- A/B, grid tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SPP=256 AB_ROUNDS=3 AB_SPC=0 AB_SCENES=final_ned timeout -k 10 300 \
    python -u tools/ab.py ab/rt.so ab/rt.so:RTOW_RUNTREE=3 ab/rtw.so > gpurun_out/ab_rtw.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_grid.py tests/test_gpu_fullres.py tests/test_gpu_fuzz.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/gputests_rtw.log 2>&1 || exit $?
