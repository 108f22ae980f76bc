set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests_r03b.log 2>&1 || exit $?
AB_SCENES=random_ned AB_SPP=64 AB_ROUNDS=3 timeout -k 10 300 python tools/ab.py ab/nows.so ab/cur.so ab/m16.so ab/m32.so ab/m16r0.so ab/m1r0.so > gpurun_out/ab_ws2.log 2>&1 || exit $?
AB_SCENES=random_ned AB_SPP=1024 AB_ROUNDS=2 AB_SPC=0 timeout -k 10 300 python tools/ab.py ab/nows.so:RTOW_AUTO_SPC=16 ab/nows.so:RTOW_AUTO_SPC=32 ab/nows.so:RTOW_AUTO_SPC=64 > gpurun_out/ab_spc.log 2>&1 || exit $?
for sc in 16 64; do RTOW_AUTO_SPC=$sc RS_SPC=0 RS_WORLDS=1,8 timeout -k 10 200 python tools/rank_share.py > gpurun_out/rank_share_spc$sc.log 2>&1 || exit $?; done
cd /tmp
for sc in 16 64; do RTOW_AUTO_SPC=$sc timeout -k 10 -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc_spc$sc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/pmc_spc$sc.log 2>&1 || exit $?; done
