set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pp_persistent" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python tools/gemm_ab.py --modes 6,10 --rounds 5 > $O/ab.jsonl 2> $O/ab.err
