import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cluster_anywhere_amd.ops.flash import flash_attention_qkv
B, T, H, D = 8, 1024, 25, 64
qkv = torch.randn(B, T, 3 * H * D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
for _ in range(3):
    o = flash_attention_qkv(qkv, H, True)
    o.backward(torch.ones_like(o))
torch.cuda.synchronize()
