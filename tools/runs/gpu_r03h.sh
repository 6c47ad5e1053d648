set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03h
timeout -k 10 200 python tools/gemm_ab.py --modes 7,8,9 --shapes sq4096,sq8192,gpt2_fc,7B_qkv_P1 --rounds 5 > gpurun_out/r03h/w4d_sq.jsonl 2> gpurun_out/r03h/w4d.err || exit $?
timeout -k 10 400 python tools/tp_gemm_table.py --modes s7,s9 --lmhead --rounds 5 > gpurun_out/r03h/w4d_tp.jsonl 2>> gpurun_out/r03h/w4d.err || exit $?
bash tools/gpu_pmc.sh gemm256s9 > gpurun_out/r03h/pmc.log 2>&1
