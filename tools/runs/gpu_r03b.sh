set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
timeout -k 10 400 python tools/tp_gemm_table.py --modes s7,s8,s9,s10 --lmhead --rounds 7 > gpurun_out/r03b/bsplit.jsonl 2> gpurun_out/r03b/bsplit.err || exit $?
timeout -k 10 200 python tools/gemm_ab.py --modes 7,8,9,10 --shapes sq8192,sq4096,gpt2_fc --rounds 7 > gpurun_out/r03b/bsplit_sq.jsonl 2>> gpurun_out/r03b/bsplit.err || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_comm_gpu.py -k "ranks_stay_identical or tp_forward_ranks or shard_as" > gpurun_out/r03b/pytest.log 2>&1
