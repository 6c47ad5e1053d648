set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_comm_gpu.py tests/test_kernels_gpu.py -k "tp_ or concurrent" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python tools/diag/tp_overlap_probe.py --P 8 --chunks 1,2,4 --streams 0,1 > $O/probe_p8.jsonl 2> $O/probe_p8.err || exit $?
timeout -k 10 400 python tools/diag/tp_overlap_probe.py --P 4 --chunks 1,2 --streams 0,1 > $O/probe_p4.jsonl 2> $O/probe_p4.err || exit $?
timeout -k 10 400 python tools/diag/tp_overlap_probe.py --P 2 --chunks 1,2 --streams 0,1 > $O/probe_p2.jsonl 2> $O/probe_p2.err
