# round 4, final build: every BASELINE config at full size and whole-frame
# parity of every config (tools/round_check.sh r04 configs,validate)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/round_check.sh r04 configs,validate
