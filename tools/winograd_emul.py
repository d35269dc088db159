"""CPU emulation (diagnostic, no GPU): operand-rounding error of a Winograd F(2x2,3x3) form of
the adapters' 3x3 convs against the direct implicit GEMM, both with the kernels' two-plane
split-bf16 operands (hi*hi + hi*lo + lo*hi, fp32 accumulation), on the ViT adapter.7 shape
(256 -> 128 channels; a 32 x 32 crop of the map, seeded random activations of the model's
scale). Reports max |y - y_fp64| / sum|x||w| per output (Winograd).

    python tools/winograd_emul.py
"""
import torch
import torch.nn.functional as F

torch.manual_seed(0)
torch.set_num_threads(8)


def split2(t):
    """two bf16 planes (RNE): the kernels' precision-0 operand split"""
    hi = t.to(torch.bfloat16).float()
    lo = (t - hi).to(torch.bfloat16).float()
    return hi, lo


def mm3(a, b):
    """a @ b with both operands split: lo*hi + hi*lo + hi*hi, fp32 accumulate"""
    ah, al = split2(a)
    bh, bl = split2(b)
    return al @ bh + ah @ bl + ah @ bh


Ci, Co, H, W = 256, 128, 32, 32
x = torch.randn(1, Ci, H, W) * 0.5
w = torch.randn(Co, Ci, 3, 3) / (Ci * 9) ** 0.5
ref = F.conv2d(x.double(), w.double(), padding=1)
den = F.conv2d(x.double().abs(), w.double().abs(), padding=1)

# direct: im2col GEMM with split operands
cols = F.unfold(x, 3, padding=1)                       # [1, Ci*9, H*W]
yd = mm3(w.reshape(Co, -1), cols[0]).reshape(1, Co, H, W)

# Winograd F(2x2, 3x3): Y = A^T [ (G g G^T) . (B^T d B) ] A, transforms in fp32 (weights in fp64
# then rounded once to fp32, as a pack-time transform would), the 16 per-position GEMMs split
Bt = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float32)
G = torch.tensor([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], dtype=torch.float64)
At = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float32)
U = (G @ w.double() @ G.T).float()                    # [Co, Ci, 4, 4]
xp = F.pad(x, (1, 1, 1, 1))[0]                         # [Ci, H+2, W+2]
tiles = xp.unfold(1, 4, 2).unfold(2, 4, 2)             # [Ci, H/2, W/2, 4, 4]
V = Bt @ tiles @ Bt.T                                  # fp32 input transform
M = torch.empty(Co, H // 2, W // 2, 4, 4)
for i in range(4):
    for j in range(4):
        M[..., i, j] = mm3(U[:, :, i, j], V[..., i, j].reshape(Ci, -1)).reshape(Co, H // 2, W // 2)
Yt = At @ M @ At.T                                     # [Co, H/2, W/2, 2, 2]
yw = Yt.permute(0, 1, 3, 2, 4).reshape(1, Co, H, W)

cpu = F.conv2d(x, w, padding=1)
for name, y in (("direct, 2-plane bf16 (shipped)", yd), ("Winograd F(2x2,3x3), 2-plane bf16", yw),
                ("CPU fp32 conv", cpu)):
    e = ((y.double() - ref).abs() / den).max().item()
    print(f"{name:38s} max |y - y64| / sum|x||w| = {e:.2e}")
