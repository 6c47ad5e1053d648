set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O/tp $O/tp_bw
TP="python -m distributed_llm_backend_benchmark_amd.cli.run_tp --config config/7b_config.yaml --backend rccl"
timeout -k 10 200 python tools/diag/pp_tile_overhead.py > $O/pp_tile_overhead_first.jsonl 2> $O/pp_tile_overhead_first.err || exit $?
for P in 2 4 8; do
  timeout -k 10 300 $TP --shard-as $P --overlap-chunks 2 --emulate-busbw 300 --output-dir $O/tp_bw > $O/tp_shard${P}_ov2_bw300.log 2>&1 || exit $?
  timeout -k 10 300 $TP --shard-as $P --overlap-chunks 2 --emulate-busbw 100 --output-dir $O/tp > $O/tp_shard${P}_ov2_bw100.log 2>&1 || exit $?
  timeout -k 10 300 $TP --shard-as $P --emulate-busbw 100 --output-dir $O/tp > $O/tp_shard${P}_bw100.log 2>&1 || exit $?
done
timeout -k 10 200 python tools/diag/pp_tile_overhead.py > $O/pp_tile_overhead.jsonl 2> $O/pp_tile_overhead.err
