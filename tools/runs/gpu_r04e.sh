# round 4: the whole GPU suite on the current tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
