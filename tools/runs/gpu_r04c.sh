# round 4: 256x192 NT tiles — numerics, then the GEMM table (7B TP shapes P=1..8 + GPT-2 fwd)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "192 or gemm_plain or gemm_epilogues" > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python tools/tp_gemm_table.py --ps 1,2,4,8 --gpt2 --modes auto,v192 > $O/gemm_table.jsonl 2> $O/gemm_table.err || exit $?
