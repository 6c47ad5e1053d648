set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O/tp
TP="python -m distributed_llm_backend_benchmark_amd.cli.run_tp --config config/7b_config.yaml --backend rccl --emulate-busbw 300 --output-dir $O/tp"
for P in 8 4 2; do
  timeout -k 10 300 $TP --shard-as $P --overlap-chunks 2 --graph > $O/p${P}_ov2_graph.log 2>&1 || exit $?
  timeout -k 10 300 $TP --shard-as $P --overlap-chunks 2 --chunk-streams > $O/p${P}_ov2cs.log 2>&1 || exit $?
done
