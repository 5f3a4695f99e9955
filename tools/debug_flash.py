import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops import kernels
from cluster_anywhere_amd.ops.attention import attention_ref
C = kernels()
B, T, H, D = 1, 128, 1, 64
torch.manual_seed(0)
qkv = torch.randn(B, T, 3 * H * D, device="cuda", dtype=torch.bfloat16)
out, lse = C.flash_attn_fwd(qkv, H, True)
dout = torch.randn_like(out)
dqkv = torch.full_like(qkv, 7.0)
delta = torch.full_like(lse, 3.0)
torch.cuda.synchronize()
# call kernels through the binding (it allocates its own dqkv)
g = C.flash_attn_bwd(qkv, out, dout, lse, H, True)
torch.cuda.synchronize()
qf = qkv.float().requires_grad_()
q, k, v = qf.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4).unbind(0)
ref = attention_ref(q, k, v, True).transpose(1, 2).reshape(B, T, H * D)
ref.backward(dout.float())
gr = qf.grad.view(B, T, 3, H, D); gg = g.view(B, T, 3, H, D).float()
for i, n in enumerate("qkv"):
    a, b = gg[:, :, i], gr[:, :, i]
    print(n, "rel", ((a - b).norm() / b.norm()).item(), "nz", (a != 0).sum().item(), "absmax", a.abs().max().item(), b.abs().max().item())
print("lse ok", torch.allclose(lse, torch.logsumexp((q @ k.transpose(-1,-2)/8).masked_fill(~torch.ones(T,T,dtype=torch.bool,device='cuda').tril(), float('-inf')), -1), atol=1e-2))
print("row 5 dq", gg[0, 5, 0, 0, :8], gr[0, 5, 0, 0, :8])
