set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03d
timeout -k 10 400 python -u tools/diag/ddp_tail_factors.py 300 > gpurun_out/r03d/factors300.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/diag/ddp_tail_factors.py 100 > gpurun_out/r03d/factors100.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_comm_gpu.py -k "fenced" > gpurun_out/r03d/pytest.log 2>&1
