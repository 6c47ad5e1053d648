set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
A="--P 8 --chunks 1,2 --streams 0 --variants both"
timeout -k 10 300 python tools/diag/tp_overlap_probe.py $A --init-pg --pg-eager > $O/eager.jsonl 2> $O/eager.err || exit $?
timeout -k 10 300 python tools/diag/tp_overlap_probe.py $A --init-pg > $O/lazy.jsonl 2> $O/lazy.err || exit $?
mkdir -p $O/tp
timeout -k 10 300 python -m distributed_llm_backend_benchmark_amd.cli.run_tp --config config/7b_config.yaml --shard-as 8 --overlap-chunks 2 --emulate-busbw 300 --backend rccl --output-dir $O/tp > $O/tp.log 2>&1
