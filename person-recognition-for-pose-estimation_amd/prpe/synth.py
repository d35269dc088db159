"""Deterministic synthetic frames and weights (no network, no checkpoints available).

Every tensor is drawn from a counter-based splitmix64 stream, so any machine
(this container, the GPU box) regenerates bit-identical tensors without shipping them:

    u64[i] = splitmix64(key_hash(seed, name) + i)        i = 0 .. numel-1
    unit[i] = (u64[i] >> 40) * 2**-24                     exact float32 in [0, 1)

Weights follow the state_dict layout of the reference ``CombinedModel``
(training/modify_models.py:462-534; key list in ``prpe.arch.state_dict_spec``).
BatchNorm running statistics are *calibrated* values shipped in
``prpe/data/bn_calib_seed1.npz`` (made once by ``oracle/make_calibration.py`` from the
seed-1 weights), so activations stay O(1) through all ~300 layers.
"""
from __future__ import annotations

import hashlib
import os

import numpy as np
import torch

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_DATA = os.path.join(os.path.dirname(__file__), "data")
CALIB_FILE = os.path.join(_DATA, "bn_calib_seed1.npz")
WEIGHT_SEED = 1
INPUT_SEED = 0


def _key_hash(seed: int, name: str) -> int:
    h = hashlib.blake2b(f"{seed}:{name}".encode(), digest_size=8).digest()
    return int.from_bytes(h, "little")


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform(seed: int, name: str, shape, lo: float = 0.0, hi: float = 1.0) -> torch.Tensor:
    """float32 tensor, U[lo, hi), deterministic in (seed, name, shape)."""
    n = int(np.prod(shape)) if len(shape) else 1
    out = np.empty(n, dtype=np.float32)
    base = np.uint64(_key_hash(seed, name))
    chunk = 1 << 24
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        with np.errstate(over="ignore"):
            ctr = base + np.arange(s, e, dtype=np.uint64)
        u = (splitmix64(ctr) >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
        out[s:e] = u
    if lo != 0.0 or hi != 1.0:
        out = np.float32(lo) + out * np.float32(hi - lo)
    return torch.from_numpy(out.reshape(shape))


def frames(batch: int, height: int = 640, width: int = 640, seed: int = INPUT_SEED,
           name: str = "frames") -> torch.Tensor:
    """Synthetic frames U[0,1) [B,3,H,W] float32 (BASELINE.md 'Synthetic inputs')."""
    return uniform(seed, f"{name}:{batch}x{height}x{width}", (batch, 3, height, width))


def frame_rows(batch: int, rows, height: int = 640, width: int = 640, seed: int = INPUT_SEED,
               name: str = "frames") -> torch.Tensor:
    """``frames(batch, ...)[rows]`` bit for bit, generating only those frames (the stream is
    counter-based: frame f is elements f*3*H*W .. (f+1)*3*H*W of the same stream)."""
    per = 3 * height * width
    base = np.uint64(_key_hash(seed, f"{name}:{batch}x{height}x{width}"))
    out = np.empty((len(rows), per), dtype=np.float32)
    for j, f in enumerate(rows):
        if not 0 <= f < batch:
            raise IndexError(f"frame {f} outside a batch of {batch}")
        with np.errstate(over="ignore"):
            ctr = base + np.arange(f * per, (f + 1) * per, dtype=np.uint64)
        out[j] = (splitmix64(ctr) >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
    return torch.from_numpy(out.reshape(len(rows), 3, height, width))


def _is_residual_branch_tail(name: str) -> bool:
    return (name.endswith("bn3.weight")                                   # ResNet bottleneck
            or name.endswith("res_layer.5.weight")                        # IR-50 BasicBlockIR
            or (".yolo." in name and ".res_m." in name and name.endswith("conv2.norm.weight"))  # yolopt Residual
            or name.endswith("conv1.conv2.norm.weight")                   # PSA attention out
            or name.endswith("conv2.1.norm.weight"))                      # PSA FFN out


def _init_for(name: str, shape) -> tuple[float, float] | str:
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":
        return "zero_int"
    if name.endswith("head.dfl.conv.weight"):
        return "arange"
    if leaf in ("running_mean",):
        return (-0.1, 0.1)
    if leaf in ("running_var",):
        return (0.8, 1.2)
    if name.endswith("ada_face.head.t"):
        return "zero"
    if name.endswith("ada_face.head.batch_mean"):
        return "const20"
    if name.endswith("ada_face.head.batch_std"):
        return "const100"
    if leaf == "position_embeddings":
        return (-0.2, 0.2)
    if ".yolo.head.cls." in name and name.split(".yolo.head.cls.")[1].split(".")[1] == "4":
        # final 1-class logit conv: keep sigmoid scores in (1e-3, 0.5), unsaturated, so the
        # NMS order is tie-free (exact float ties would make the upstream order unspecified)
        return (-0.02, 0.02) if leaf == "weight" else (-4.5, -3.5)
    if _is_residual_branch_tail(name):
        # last BN of a residual branch: small gamma (torchvision zero_init_residual / Fixup
        # style). Random deep nets with O(1) residual branches are chaotic (2^-17 weight
        # noise moves the trunk output by 3e-3 relative); trained nets are not. With this
        # the model's sensitivity is ~80x lower (measured, DESIGN.md "Conditioning").
        return (0.05, 0.25)
    if len(shape) == 1:
        # BN / LN affine, PReLU slopes, biases.  Distinguish by sibling naming.
        if "layernorm" in name:
            return (0.8, 1.2) if leaf == "weight" else (-0.1, 0.1)
        if leaf == "weight":
            return "affine_or_prelu"
        return (-0.1, 0.1)
    fan_in = int(np.prod(shape[1:]))
    b = float(np.sqrt(3.0 / fan_in))
    return (-b, b)


def make_state_dict(spec, seed: int = WEIGHT_SEED, calib: bool = True,
                    skip=("ada_face.head.kernel",)) -> dict[str, torch.Tensor]:
    """Build a state_dict for ``spec`` = [(name, shape, kind)], kind in
    {'conv','linear','bn','prelu','ln','bias','other'} (see prpe.arch)."""
    sd: dict[str, torch.Tensor] = {}
    for name, shape, kind in spec:
        shape = tuple(shape)
        if name in skip:
            continue
        init = _init_for(name, shape)
        if init == "zero_int":
            sd[name] = torch.zeros((), dtype=torch.int64)
        elif init == "arange":
            sd[name] = torch.arange(shape[1], dtype=torch.float32).view(shape)
        elif init == "zero":
            sd[name] = torch.zeros(shape)
        elif init == "const20":
            sd[name] = torch.full(shape, 20.0)
        elif init == "const100":
            sd[name] = torch.full(shape, 100.0)
        elif init == "affine_or_prelu":
            if kind == "prelu":
                sd[name] = uniform(seed, name, shape, 0.1, 0.4)
            else:
                sd[name] = uniform(seed, name, shape, 0.6, 1.4)
        else:
            lo, hi = init
            sd[name] = uniform(seed, name, shape, lo, hi)
    if calib:
        if not os.path.exists(CALIB_FILE):
            raise FileNotFoundError(f"BN calibration file missing: {CALIB_FILE}")
        with np.load(CALIB_FILE, allow_pickle=False) as z:
            for k in z.files:
                if k in sd:
                    sd[k] = torch.from_numpy(np.array(z[k], dtype=np.float32))
    return sd


def head_kernel(seed: int = WEIGHT_SEED) -> torch.Tensor:
    """ada_face.head.kernel [512, 85742] (training head; only the eval logits GEMM reads it)."""
    return uniform(seed, "ada_face.head.kernel", (512, 85742), -0.05, 0.05)
