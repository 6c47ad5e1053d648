set -u
cd /root/repo
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 20 --warmup 5 --output gpurun_out/gpt2.json > gpurun_out/gpt2.log 2>&1 || exit $?
tail -2 gpurun_out/gpt2.log
bash tools/gpu_profile.sh gpt2
