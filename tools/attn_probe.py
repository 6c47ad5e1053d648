"""Probe torch's ROCm flash-attention ops: output layout and the logsumexp format."""
import math

import torch
import torch.nn.functional as F

B, T, H, D = 2, 256, 4, 64
qkv = torch.randn(B, T, 3 * H * D, device="cuda", dtype=torch.bfloat16)
q, k, v = qkv.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4).unbind(0)
o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
print("sdpa out stride", o.stride(), "transposed-contig", o.transpose(1, 2).is_contiguous())
r = torch.ops.aten._scaled_dot_product_flash_attention(q, k, v, 0.0, True, False)
print("flash fwd returns", len(r), [getattr(x, "shape", x) for x in r])
lse = r[1]
s = (q.float() @ k.float().transpose(-1, -2)) / math.sqrt(D)
mask = torch.ones(T, T, device="cuda", dtype=torch.bool).triu(1)
s = s.masked_fill(mask, float("-inf"))
ref_ln = torch.logsumexp(s, -1)
print("lse dtype", lse.dtype, "shape", lse.shape, "stride", lse.stride())
print("max |lse - ln-sum-exp|", float((lse - ref_ln).abs().max()),
      "max |lse - log2-sum-exp|", float((lse - ref_ln / math.log(2)).abs().max()))
go = torch.randn_like(o)
g = torch.ops.aten._scaled_dot_product_flash_attention_backward(
    go, q, k, v, r[0], r[1], r[2], r[3], r[4], r[5], 0.0, True, r[6], r[7])
print("bwd returns", [x.shape for x in g], [x.stride() for x in g])
