set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
timeout -k 10 500 python -u tools/overlap_trap.py --out gpurun_out/r03c/trap > gpurun_out/r03c/trap.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/ddp_tail.py --out gpurun_out/r03c/ddp_tail.jsonl > gpurun_out/r03c/ddp_tail.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_comm_gpu.py -k "ranks_stay_identical or tp_forward_ranks or shard_as" > gpurun_out/r03c/pytest.log 2>&1
