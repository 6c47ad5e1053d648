# overlapped TP forward: tests, shard projections with/without link time, kernel stats
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R${PYTHONPATH:+:$PYTHONPATH}
O=$R/gpurun_out/r03l
mkdir -p $O/tp $O/tp_bw
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_comm_gpu.py -k "tp_" > $O/pytest_tp.log 2>&1 || exit $?
TP="python -m distributed_llm_backend_benchmark_amd.cli.run_tp --config config/7b_config.yaml --backend rccl"
for P in 2 4 8; do
  for N in 2 4; do
    timeout -k 10 300 $TP --shard-as $P --overlap-chunks $N --output-dir $O/tp > $O/tp_shard${P}_ov$N.log 2>&1 || exit $?
    timeout -k 10 300 $TP --shard-as $P --overlap-chunks $N --emulate-busbw 300 --output-dir $O/tp_bw > $O/tp_shard${P}_ov${N}_bw300.log 2>&1 || exit $?
  done
  timeout -k 10 300 $TP --shard-as $P --emulate-busbw 300 --output-dir $O/tp_bw > $O/tp_shard${P}_bw300.log 2>&1 || exit $?
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tp7b -o tp7b -- python3 -m distributed_llm_backend_benchmark_amd.cli.run_tp --config $R/config/7b_config.yaml --backend rccl --output-dir $O/tp_prof > $O/prof_tp7b.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tp7b_shard4 -o tp7b_shard4 -- python3 -m distributed_llm_backend_benchmark_amd.cli.run_tp --config $R/config/7b_config.yaml --backend rccl --shard-as 4 --output-dir $O/tp_prof > $O/prof_tp7b_shard4.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gpt2 -o gpt2 -- python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 10 --warmup 3 > $O/prof_gpt2.log 2>&1
