"""
TEST INFRASTRUCTURE ONLY (never imported by the product path): a plain-Python restatement of the
device minibatch row order of ``mininf_amd/csrc/minibatch.hip`` (``mi_minibatch_rows``), used by
the tests as the checker of the kernel's rows.

What it stands in for: the reference draws minibatches with a host ``DataLoader(TensorDataset(X,
y), batch_size, shuffle=True)`` (``examples/minibatch.md:78``), i.e. torch's ``RandomSampler``
(a ``torch.randperm`` per epoch). That random order cannot be reproduced bit for bit on the
device (hard part (b): RNG streams differ), so the engine defines its own
order -- a keyed Feistel permutation per epoch -- and this restatement pins that definition. The
properties the reference's loader has and the tests check are: every epoch visits every row
exactly once, batches have ``batch_size`` rows (the last one possibly fewer unless
``drop_last``), and the order changes from epoch to epoch.
"""
from __future__ import annotations

from typing import List

M32 = 0xFFFFFFFF
ROUNDS = 4


def round_fn(x: int, key: int) -> int:
    """murmur3's 32-bit finaliser of x ^ key (minibatch.hip round_fn)."""
    x = (x ^ key) & M32
    x = (x * 0xCC9E2D51) & M32
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & M32
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & M32
    x ^= x >> 16
    return x


def feistel_half(n: int) -> int:
    bits = 2
    while bits < 62 and (1 << bits) < n:
        bits += 1
    return (bits + 1) // 2


def keys(seed: int, epoch: int) -> List[int]:
    s = (seed ^ (seed >> 32)) & M32
    e = round_fn(epoch & M32, ((epoch >> 32) + 0x7F4A7C15) & M32)
    return [round_fn(s ^ ((q * 0x9E3779B9) & M32), e) for q in range(ROUNDS)]


def feistel(x: int, half: int, k: List[int]) -> int:
    mask = (1 << half) - 1
    left, right = x >> half, x & mask
    for q in range(ROUNDS):
        left, right = right, left ^ (round_fn(right & M32, k[q]) & mask)
    return (left << half) | right


def batch_rows(counter: int, n: int, batch: int, batches: int, shuffle: bool, seed: int,
               count: int) -> List[int]:
    """rows[j], j < count, of the batch drawn at counter value `counter`."""
    epoch, b = divmod(counter, batches)
    half = feistel_half(n)
    k = keys(seed & ((1 << 64) - 1), epoch)
    out = []
    for j in range(count):
        x = b * batch + j
        if shuffle:
            x = feistel(x, half, k)
            while x >= n:
                x = feistel(x, half, k)
        out.append(x)
    return out
