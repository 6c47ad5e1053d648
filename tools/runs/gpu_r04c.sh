# round 4: 256x192 NT tiles and NT split-K — numerics, then the GEMM table (7B TP P=1..8 + GPT-2)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
true
timeout -k 10 400 python tools/tp_gemm_table.py --ps 1,2,4,8 --gpt2 --modes auto,v192,sk,sk192 > $O/gemm_table.jsonl 2> $O/gemm_table.err || exit $?
