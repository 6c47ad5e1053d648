set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03j
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r03j/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python bench.py > gpurun_out/r03j/bench.json 2> gpurun_out/r03j/bench.err
