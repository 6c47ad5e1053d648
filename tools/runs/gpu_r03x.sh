set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 400 python tools/diag/ddp_tail_factors.py 100 > $O/factors_lazy_100.log 2> $O/factors_lazy_100.err || exit $?
DLBB_RCCL_EAGER_INIT=1 timeout -k 10 400 python tools/diag/ddp_tail_factors.py 100 > $O/factors_eager_100.log 2> $O/factors_eager_100.err
