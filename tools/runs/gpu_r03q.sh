set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O/a $O/b $O/d
TP="python -m distributed_llm_backend_benchmark_amd.cli.run_tp --config config/7b_config.yaml --shard-as 8 --overlap-chunks 2 --emulate-busbw 300"
timeout -k 10 300 $TP --backend rccl --output-dir $O/a > $O/a.log 2>&1 || exit $?
timeout -k 10 300 $TP --backend gloo --device cuda --output-dir $O/b > $O/b.log 2>&1 || exit $?
timeout -k 10 300 $TP --backend rccl --warmup 3 --iters 5 --output-dir $O/d > $O/d.log 2>&1 || exit $?
timeout -k 10 300 python tools/diag/tp_overlap_probe.py --P 8 --chunks 2 --streams 0 --variants both --init-pg > $O/c.jsonl 2> $O/c.err
