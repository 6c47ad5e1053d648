set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
A="--P 8 --chunks 2 --streams 0 --variants both"
timeout -k 10 300 python tools/diag/tp_overlap_probe.py $A --init-pg --pg-eager > $O/eager.jsonl 2> $O/eager.err || exit $?
timeout -k 10 300 python tools/diag/tp_overlap_probe.py $A --init-pg > $O/lazy.jsonl 2> $O/lazy.err || exit $?
NCCL_DEBUG=INFO timeout -k 10 300 python tools/diag/tp_overlap_probe.py $A --init-pg --pg-eager > $O/eager_dbg.jsonl 2> $O/eager_dbg.err
