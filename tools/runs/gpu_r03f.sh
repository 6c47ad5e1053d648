set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03f
timeout -k 10 200 python tools/gemm_ab.py --modes 7,8 --shapes sq4096,sq8192,gpt2_fc --rounds 5 > gpurun_out/r03f/w4_sq.jsonl 2> gpurun_out/r03f/w4.err || exit $?
timeout -k 10 400 python tools/tp_gemm_table.py --modes s7,s8 --lmhead --rounds 5 > gpurun_out/r03f/w4_tp.jsonl 2>> gpurun_out/r03f/w4.err
