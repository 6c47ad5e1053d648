set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03a
timeout -k 10 300 python tools/tp_gemm_table.py --modes auto,t128,t256 --lmhead --rounds 5 > gpurun_out/r03a/table.jsonl 2> gpurun_out/r03a/table.err || exit $?
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "split" tests/test_comm_gpu.py -k "split or calibration or ddp or bench_py_world1 or registered" > gpurun_out/r03a/pytest.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03a/prof -o run -- python $GRAFT_REPO_ROOT/tools/tp_gemm_table.py --modes auto --rounds 1 --iters 3 > $GRAFT_REPO_ROOT/gpurun_out/r03a/prof.log 2>&1
