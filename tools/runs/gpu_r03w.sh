set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_comm_gpu.py -k "gemm or linear or tp_ or concurrent" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python tools/gemm_ab.py --modes 7,10 --rounds 5 > $O/ab.jsonl 2> $O/ab.err || exit $?
timeout -k 10 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2.json > $O/gpt2.log 2>&1 || exit $?
DLBB_GEMM_PERSIST=0 timeout -k 10 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2_nopersist.json > $O/gpt2_nopersist.log 2>&1 || exit $?
TP="python -m distributed_llm_backend_benchmark_amd.cli.run_tp --config config/7b_config.yaml --backend rccl"
for P in 8 4 2; do
  mkdir -p $O/tp_eager $O/tp_graph
  timeout -k 10 300 $TP --shard-as $P --overlap-chunks 2 --emulate-busbw 300 --output-dir $O/tp_eager > $O/p${P}_ov2.log 2>&1 || exit $?
  timeout -k 10 300 $TP --shard-as $P --emulate-busbw 300 --output-dir $O/tp_eager > $O/p${P}.log 2>&1 || exit $?
  timeout -k 10 300 $TP --shard-as $P --overlap-chunks 2 --emulate-busbw 300 --graph --output-dir $O/tp_graph > $O/p${P}_ov2_graph.log 2>&1 || exit $?
  timeout -k 10 300 $TP --shard-as $P --emulate-busbw 300 --graph --output-dir $O/tp_graph > $O/p${P}_graph.log 2>&1 || exit $?
done
