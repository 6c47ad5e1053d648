# TP 7B per-rank projection + final kernel stats for TP 7B and GPT-2 DDP
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03k
mkdir -p $O/tp $O/tp_bw
TP="python -m distributed_llm_backend_benchmark_amd.cli.run_tp --config config/7b_config.yaml --backend rccl"
timeout -k 10 300 $TP --output-dir $O/tp > $O/tp_world1.log 2>&1 || exit $?
for P in 2 4 8; do
  timeout -k 10 300 $TP --shard-as $P --output-dir $O/tp > $O/tp_shard$P.log 2>&1 || exit $?
  timeout -k 10 300 $TP --shard-as $P --emulate-busbw 300 --output-dir $O/tp_bw > $O/tp_shard${P}_bw300.log 2>&1 || exit $?
done
timeout -k 10 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2.json > $O/gpt2.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tp7b -o tp7b -- python3 -m distributed_llm_backend_benchmark_amd.cli.run_tp --config $R/config/7b_config.yaml --backend rccl --output-dir $O/tp_prof > $O/prof_tp7b.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tp7b_shard8 -o tp7b_shard8 -- python3 -m distributed_llm_backend_benchmark_amd.cli.run_tp --config $R/config/7b_config.yaml --backend rccl --shard-as 8 --output-dir $O/tp_prof > $O/prof_tp7b_shard8.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gpt2 -o gpt2 -- python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 10 --warmup 3 > $O/prof_gpt2.log 2>&1
