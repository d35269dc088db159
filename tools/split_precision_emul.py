"""CPU emulation of the split-operand GEMM schemes (diagnostics, no GPU): worst-case error per
output relative to sum |a||w|, against an fp64 reference, for a trunk-like 3x3 conv GEMM
(K = 2304, post-ReLU activations).

    python tools/split_precision_emul.py

Schemes: CPU fp32 itself; bf16 planes NP=2 (3 MFMA terms) and NP=3 (6 terms); fp16 planes
NP=2 (3 terms) with a power-of-2 scale per tensor (activations) / per output channel
(weights) that puts each maximum just under 2^15, and without scaling.
"""
import math

import torch


def split(x, dt, n):
    r = x.double().clone()
    ps = []
    for _ in range(n):
        p = r.float().to(dt).double()
        ps.append(p)
        r = r - p
    return ps


def emul(a, w, dt, n, sa=1.0, sw=None):
    N = w.shape[1]
    sw = torch.ones(N, dtype=torch.float64) if sw is None else sw
    A = split(a.double() * sa, dt, n)
    W = split(w.double() * sw, dt, n)
    acc = torch.zeros(a.shape[0], N, dtype=torch.float64)
    for i in range(n):
        for j in range(n):
            if i + j < n:
                acc += (A[i] @ W[j])            # products of planes are exact in fp64
    return acc / sa / sw


def main():
    torch.manual_seed(0)
    M, K, N = 256, 2304, 128
    for amp in (3.0, 300.0, 0.01):
        a = torch.relu(torch.randn(M, K)) * amp
        w = torch.randn(K, N) / K ** 0.5
        ref = a.double() @ w.double()
        den = a.double().abs() @ w.double().abs()
        err = lambda x: ((x - ref).abs() / den).max().item()
        e = math.frexp(a.abs().max().item())[1]
        sa = 2.0 ** (15 - e)
        sw = 2.0 ** (15 - torch.frexp(w.abs().max(0).values.double())[1].double())
        print(f"activation scale {amp}:")
        print(f"  fp32 CPU            {err((a @ w).double()):.3e}")
        print(f"  bf16 NP=2 (3 terms) {err(emul(a, w, torch.bfloat16, 2)):.3e}")
        print(f"  bf16 NP=3 (6 terms) {err(emul(a, w, torch.bfloat16, 3)):.3e}")
        print(f"  f16  NP=2 scaled    {err(emul(a, w, torch.float16, 2, sa, sw)):.3e}")
        print(f"  f16  NP=2 unscaled  {err(emul(a, w, torch.float16, 2)):.3e}")


if __name__ == "__main__":
    main()
