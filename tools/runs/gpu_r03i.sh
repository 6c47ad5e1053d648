set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03i
timeout -k 10 300 python tools/gemm_ab.py --modes 7,9,10,11,12 --shapes sq4096,sq8192,gpt2_fc,7B_qkv_P1,7B_down_P1 --rounds 5 > gpurun_out/r03i/w4dv.jsonl 2> gpurun_out/r03i/w4dv.err
