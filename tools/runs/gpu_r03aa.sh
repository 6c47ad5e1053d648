set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_streams_gpu.py tests/test_virtual_ranks_gpu.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
