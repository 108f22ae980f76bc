# Scratch GPU session (one gpurun call): the grid tests verbose, then the
# whole GPU suite.  Round-end profiles and configs: tools/round_check.sh.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_grid.py -m gpu -v -s --timeout 120 --timeout-method thread \
    > gpurun_out/grid_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gputests.log 2>&1 || exit $?
