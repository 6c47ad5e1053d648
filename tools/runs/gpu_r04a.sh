# round 4: bench.py with the BASELINE config 3-5 sections (world 1 + two-rank rehearsal), the
# DDP auto-path rehearsal, then a rocprof kernel table of the world-1 bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
S=$(date +%s); timeout -k 10 400 python bench.py > $O/bench_w1.json 2> $O/bench_w1.err || exit $?; echo "bench wall $(( $(date +%s) - S )) s" > $O/bench_wall.txt
timeout -k 10 900 $T tests/test_comm_gpu.py -k "bench_py or ddp_matches_global" > $O/tests.log 2>&1 || exit $?
