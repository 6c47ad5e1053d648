import json, os, sys, torch
sys.path.insert(0, os.getcwd())
from distributed_llm_backend_benchmark_amd.ops import _lib
from distributed_llm_backend_benchmark_amd.ops.attention import attn_fwd
lib = _lib.lib()
def t_best(fn, iters=20, rounds=6):
    best = 1e9
    for _ in range(rounds):
        fn(); torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters): fn()
        e.record(); e.synchronize()
        best = min(best, s.elapsed_time(e) / iters * 1e-3)
    return best
for B, T, H in ((16, 1024, 12), (8, 2048, 12), (4, 4096, 16)):
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda").to(torch.bfloat16)
    fl = 4.0 * B * H * T * T * 64 / 2
    res = {}
    for v in (6, 100):
        lib.dlbb_attn_set_fwd_variant(v)
        res[v] = t_best(lambda: attn_fwd(qkv, H))
    print(json.dumps({"B": B, "T": T, "H": H, **{f"v{v}_us": round(t * 1e6, 2) for v, t in res.items()},
                      **{f"v{v}_tflops": round(fl / t / 1e12, 1) for v, t in res.items()}}), flush=True)
