set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03g
timeout -k 10 200 python tools/gemm_ab.py --modes 7,8 --shapes sq4096,sq8192,gpt2_fc,7B_qkv_P1 --rounds 5 > gpurun_out/r03g/w4_sq.jsonl 2> gpurun_out/r03g/w4.err || exit $?
bash tools/gpu_pmc.sh gemm256s8 gemm256s7 blas > gpurun_out/r03g/pmc.log 2>&1
