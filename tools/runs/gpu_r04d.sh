# round 4: where a ping-pong workgroup's time goes (phase stamps) vs hipBLASLt wall
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 300 python tools/diag/pp_phases.py --nj 4,3 > $O/phases.jsonl 2> $O/phases.err || exit $?
