# round 4 (session 2): grid walk for final_ned's ground (MODE 8) and the
# bare v_min_f32 slab bound -- grid tests, A/B against the committed build,
# then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_grid.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/grid_tests.log 2>&1 || exit $?
AB_SPP=256 AB_ROUNDS=3 AB_SPC=0 AB_SCENES=final_ned,cornell,cornell_smoke,random_ned timeout -k 10 500 \
    python -u tools/ab.py ab/base.so ab/asmmin.so ab/grid.so ab/grid.so:RTOW_GRID=0 > gpurun_out/ab_grid.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gputests_grid.log 2>&1 || exit $?
