# round 4: the 4-wide tree variants (stack entries inside each lane's own
# 32-bit column now) on small frames first, then an A/B on config 2 at 256 spp
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
RTOW_WIDE_DEBUG=1 timeout -k 10 200 python -u tools/wide_smoke.py 4 3 4:1 4:16 4:32 4:48 > gpurun_out/wide_smoke_r04d.txt 2>&1 || exit $?
AB_SPP=256 AB_ROUNDS=3 AB_SPC=0 AB_SCENES=random_ned timeout -k 10 200 \
    python -u tools/ab.py ab/new.so ab/new.so:RTOW_WIDE=3 ab/new.so:RTOW_WIDE=4 ab/new.so:RTOW_WIDE=4,RTOW_SPEC=1 \
    ab/new.so:RTOW_WIDE=4,RTOW_SPEC=16 ab/new.so:RTOW_WIDE=4,RTOW_SPEC=32 > gpurun_out/ab_wide_r04d.txt 2>&1 || exit $?
