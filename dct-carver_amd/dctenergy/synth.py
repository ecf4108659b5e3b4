"""Synthetic frames for the bench and the large-size tests (torch: device memory only).

"Natural-like" RGB: clip(round(128 + 60 sin(x/17) + 40 cos(y/11)
+ N(0, 20))) per channel.  The noise is a counter-based hash of (seed, global
row, column, channel), so any rank can generate any rows of the global frame
(row bands + halos) without communication, and a frame is reproducible.
"""
import math


def _hash_uniform(idx, seed, torch):
    # splitmix64-style finaliser on int64 (wrapping arithmetic), -> (0, 1)
    # the seed's term wrapped to int64 here (torch takes ints below 2^64 and
    # wraps them the same way, so seeds that fit give the frames they always gave)
    k = (seed * 0x14057B7EF767814F + 0x2545F4914F6CDD1D) & 0xFFFFFFFFFFFFFFFF
    z = idx * 0x5851F42D4C957F2D + (k - (1 << 64) if k >= (1 << 63) else k)
    z = z ^ ((z >> 31) & 0x1FFFFFFFF)
    z = z * 0x7FB5D329728EA185
    z = z ^ ((z >> 27) & 0x1FFFFFFFFF)
    z = z * 0x2545F4914F6CDD1D
    z = z ^ ((z >> 33) & 0x7FFFFFFF)
    return ((z & 0xFFFFFF).to(torch.float32) + 0.5) / float(1 << 24)


def natural_rows(y0, nrows, w, channels=3, seed=0, device="cuda", noise=20.0):
    """uint8 tensor [nrows, w, channels] (or [nrows, w] for channels == 1) =
    rows y0 .. y0 + nrows - 1 of the global natural-like frame."""
    import torch
    y = torch.arange(y0, y0 + nrows, device=device, dtype=torch.int64).view(-1, 1, 1)
    x = torch.arange(w, device=device, dtype=torch.int64).view(1, -1, 1)
    c = torch.arange(channels, device=device, dtype=torch.int64).view(1, 1, -1)
    idx = (y * w + x) * channels + c
    u1 = _hash_uniform(2 * idx, seed, torch)
    u2 = _hash_uniform(2 * idx + 1, seed, torch)
    g = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos((2.0 * math.pi) * u2)
    base = 128.0 + 60.0 * torch.sin(x.to(torch.float32) / 17.0) + 40.0 * torch.cos(y.to(torch.float32) / 11.0)
    img = torch.clamp(torch.round(base + noise * g), 0, 255).to(torch.uint8)
    return img[..., 0].contiguous() if channels == 1 else img.contiguous()
