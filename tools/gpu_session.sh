# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests_r03c.log 2>&1 || exit $?
AB_SCENES=random_ned AB_SPP=1024 AB_ROUNDS=2 AB_SPC=0 timeout -k 10 300 python tools/ab.py ab/nows.so:RTOW_AUTO_SPC=16 ab/pm.so:RTOW_AUTO_SPC=16 ab/pm.so > gpurun_out/ab_pm.log 2>&1 || exit $?
AB_SCENES=cornell_smoke,final_ned AB_SPP=256 AB_ROUNDS=2 AB_SPC=0 timeout -k 10 300 python tools/ab.py ab/nows.so:RTOW_AUTO_SPC=16 ab/pm.so:RTOW_AUTO_SPC=16 ab/pm.so > gpurun_out/ab_pm_gen.log 2>&1 || exit $?
RS_SPC=0 RS_WORLDS=1,2,8 timeout -k 10 200 python tools/rank_share.py > gpurun_out/rank_share_pm.log 2>&1 || exit $?
timeout -k 10 200 python tools/prof_counters.py final_ned 32 > gpurun_out/prof_final_r03c.log 2>&1 || exit $?
cd /tmp
timeout -k 10 -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc_pm -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/pmc_pm.log 2>&1 || exit $?
