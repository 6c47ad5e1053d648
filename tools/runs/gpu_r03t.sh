set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
TP="python -m distributed_llm_backend_benchmark_amd.cli.run_tp --config config/7b_config.yaml --backend rccl"
for P in 8 4 2; do
  for BW in 300 100; do
    mkdir -p $O/bw$BW/eager $O/bw$BW/graph
    timeout -k 10 300 $TP --shard-as $P --overlap-chunks 2 --emulate-busbw $BW --output-dir $O/bw$BW/eager > $O/p${P}_bw${BW}_ov2.log 2>&1 || exit $?
    timeout -k 10 300 $TP --shard-as $P --overlap-chunks 2 --emulate-busbw $BW --graph --output-dir $O/bw$BW/graph > $O/p${P}_bw${BW}_ov2_graph.log 2>&1 || exit $?
    timeout -k 10 300 $TP --shard-as $P --emulate-busbw $BW --graph --output-dir $O/bw$BW/graph > $O/p${P}_bw${BW}_graph.log 2>&1 || exit $?
  done
done
