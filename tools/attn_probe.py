import torch, torch.nn.functional as F
B,T,H,D=16,1024,12,64
qkv=torch.randn(B,T,3*H*D,device='cuda',dtype=torch.bfloat16,requires_grad=True)
q,k,v=qkv.view(B,T,3,H,D).permute(2,0,3,1,4).unbind(0)
o=F.scaled_dot_product_attention(q,k,v,is_causal=True)
print("out stride", o.stride(), o.shape, "is transposed-contig:", o.transpose(1,2).is_contiguous())
print(torch.backends.cuda.flash_sdp_enabled(), torch.backends.cuda.mem_efficient_sdp_enabled())
