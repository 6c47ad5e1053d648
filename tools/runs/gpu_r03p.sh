set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
A="--P 8 --chunks 1,2 --streams 0 --variants spin,both"
timeout -k 10 300 python tools/diag/tp_overlap_probe.py $A > $O/nopg.jsonl 2> $O/nopg.err || exit $?
timeout -k 10 300 python tools/diag/tp_overlap_probe.py $A --init-pg > $O/pg.jsonl 2> $O/pg.err || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/diag/tp_overlap_probe.py $A --init-pg > $O/pg_q8.jsonl 2> $O/pg_q8.err || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/diag/tp_overlap_probe.py --P 8 --chunks 2 --streams 1 --variants spin,both > $O/nopg_q8_streams.jsonl 2> $O/nopg_q8_streams.err
