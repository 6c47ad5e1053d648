set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_streams_gpu.py tests/test_comm_gpu.py -k "streams or concurrent or ddp or tp_ or fenced" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python tools/diag/ddp_tail_factors.py 100 > $O/factors_lazy_100.log 2> $O/factors_lazy_100.err || exit $?
DLBB_RCCL_EAGER_INIT=1 timeout -k 10 400 python tools/diag/ddp_tail_factors.py 100 > $O/factors_eager_100.log 2> $O/factors_eager_100.err || exit $?
timeout -k 10 300 python tools/diag/tp_overlap_probe.py --P 8 --chunks 2 --streams 0,1 --variants both --init-pg --pg-eager > $O/tp_eager.jsonl 2> $O/tp_eager.err
