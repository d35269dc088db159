"""Inputs of the golden fixtures made by oracle/make_golden_evalsteps.py (test infrastructure
only). The fixtures store only the reference's OUTPUTS and an input checksum; tests rebuild
the inputs here, bit-identically, from the splitmix64 streams of prpe.synth.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from prpe import synth


def vitpose_pixels():
    """pixel_values U[0,1) [2,3,256,192] of golden_vitpose.npz (BASELINE config 3 input)."""
    return synth.uniform(0, "pixel_values:2x256x192", (2, 3, 256, 192))


def flip_inputs():
    """(heat, heat_flipped) [3,17,64,48] of golden_flip.npz."""
    return (synth.uniform(31, "flip_heat", (3, 17, 64, 48), -1.0, 3.0),
            synth.uniform(31, "flip_heat_flipped", (3, 17, 64, 48), -1.0, 3.0))


def facerec_inputs(B=6, C=1000):
    """(emb [B,512], kernel [512,C], labels [B]) of golden_facerec.npz."""
    emb = synth.uniform(41, "facerec_emb", (B, 512), -1.0, 1.0)
    emb[2] *= 1e-3                                     # F.normalize: any norm
    kernel = synth.uniform(41, "facerec_kernel", (512, C), -0.05, 0.05)
    labels = (synth.uniform(41, "facerec_labels", (B,)) * C).long()
    # two rows classifiable: their embedding is the normalised kernel column of the label
    kn = F.normalize(kernel)
    for b in (0, 3):
        emb[b] = kn[:, labels[b]] * 3.0
    return emb, kernel, labels
