set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or linear" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python tools/gemm_ab.py --modes 7,10 --rounds 5 > $O/ab.jsonl 2> $O/ab.err || exit $?
timeout -k 10 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2.json > $O/gpt2.log 2>&1 || exit $?
DLBB_GEMM_PERSIST=0 timeout -k 10 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2_nopersist.json > $O/gpt2_nopersist.log 2>&1
