"""Reference point (GPU box, measurement only): the rate of the platform library GEMM
(torch.matmul on bf16 -> hipBLASLt) on this model's GEMM shapes, with K tripled as the 3-term
split would need (C = [A_hi | A_hi | A_lo] [B_hi ; B_lo ; B_hi]). Not on the product path: it says
how far the hand-written kernels are from what the chip does on a plain bf16 GEMM of the same
executed size.

    python tools/gemm_ceiling.py
"""
import torch

SHAPES = [("vit fc1", 49152, 768, 3072), ("vit fc2", 49152, 3072, 768), ("vit qkv", 49152, 768, 2304),
          ("vit proj", 49152, 768, 768), ("yolo adapter.7", 6553600, 512, 256),
          ("trunk l3 conv1", 409600, 1024, 256), ("trunk l3 conv3", 409600, 256, 1024)]


def timed(fn, it=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def main():
    g = torch.Generator("cuda").manual_seed(0)
    for name, M, K, N in SHAPES:
        for kx in (1, 3):
            Kx = K * kx
            a = torch.randn(M, Kx, device="cuda", dtype=torch.bfloat16, generator=g)
            b = torch.randn(Kx, N, device="cuda", dtype=torch.bfloat16, generator=g)
            ms = timed(lambda: torch.matmul(a, b))
            tf = 2 * M * N * Kx / ms / 1e9
            print(f"{name:16s} M={M:8d} K={Kx:5d} N={N:5d} bf16 hipBLASLt {ms:8.3f} ms  {tf:7.1f} TF/s executed"
                  f"  (= {2 * M * N * K / ms / 1e9:6.1f} TF/s algorithmic at {kx} term{'s' if kx > 1 else ''})",
                  flush=True)
            del a, b


if __name__ == "__main__":
    main()
