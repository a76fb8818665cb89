"""Multi-GPU sharding of a signature batch: one process per GPU
(torch.distributed, backend "nccl" = RCCL over xGMI), contiguous 64-aligned
shards, one all-gather of the packed verdict bitmaps.

Signatures are independent, so there is no data-path collective: each rank
verifies its shard on its own device; the only exchange is the final
all-gather that gives every rank the job's full verdict vector (the caller --
blocksync / light-client replay -- needs it to replay the reference loop).
Shard boundaries are multiples of 64 so a rank's bitmap words never straddle
another rank's signatures and the gathered words ARE the global bitmap.
"""
from __future__ import annotations

import numpy as np


def shard_size(n: int, world: int) -> int:
    """Signatures per rank: ceil(n / world) rounded up to a multiple of 64."""
    per = -(-n // world) if world else n
    return -(-per // 64) * 64


def shard_range(n: int, world: int, rank: int):
    s = shard_size(n, world)
    lo = min(n, rank * s)
    hi = min(n, lo + s)
    return lo, hi


def pack_bitmap(valid: np.ndarray, words: int | None = None) -> np.ndarray:
    """uint8 verdicts -> uint64 words, bit i%64 of word i//64 (the kernel's ballot layout)."""
    v = np.asarray(valid, dtype=np.uint8) != 0
    n = v.size
    w = -(-n // 64) if words is None else words
    padded = np.zeros(w * 64, dtype=np.uint8)
    padded[:n] = v
    return np.packbits(padded, bitorder="little").view(np.uint64)


def unpack_bitmap(words: np.ndarray, n: int) -> np.ndarray:
    return np.unpackbits(np.ascontiguousarray(words, dtype=np.uint64).view(np.uint8), bitorder="little")[:n]


def gather_bitmaps(local_words, n: int, world: int, group=None):
    """All-gather each rank's (padded) bitmap words; returns the global words
    (ceil(n/64)) as a tensor on the input's device. local_words: int64 tensor
    of shard_size(n, world) // 64 words."""
    import torch
    import torch.distributed as dist

    per = shard_size(n, world) // 64
    if local_words.numel() != per:
        raise ValueError(f"rank bitmap must have {per} words, got {local_words.numel()}")
    out = torch.empty(world * per, dtype=local_words.dtype, device=local_words.device)
    dist.all_gather_into_tensor(out, local_words.contiguous(), group=group)
    return out[: -(-n // 64)]


def verify_sharded(ctx, pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, msg_off: np.ndarray, mode: int,
                   world: int, rank: int, device=None, group=None):
    """Blocksync / light-client replay shape (BASELINE.json configs[2]): a
    global host batch; this rank verifies its shard on its GPU through the
    device-resident API and all ranks receive the global verdict bitmap."""
    import torch

    n = len(msg_off) - 1
    lo, hi = shard_range(n, world, rank)
    per = shard_size(n, world)
    dev = device or torch.device("cuda", torch.cuda.current_device())
    cnt = hi - lo
    m0, m1 = int(msg_off[lo]), int(msg_off[hi])
    d_pk = torch.from_numpy(np.ascontiguousarray(pk[lo:hi]).reshape(-1).copy()).to(dev)
    d_sig = torch.from_numpy(np.ascontiguousarray(sig[lo:hi]).reshape(-1).copy()).to(dev)
    d_msg = torch.from_numpy(np.concatenate([msg[m0:m1], np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy((msg_off[lo:hi + 1] - m0).astype(np.uint32).view(np.int32)).to(dev)
    d_bm = torch.zeros(per // 64, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    if cnt:
        ctx.verify_device(cnt, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(), mode,
                          0, d_bm.data_ptr(), stream.cuda_stream)
    if world > 1:
        return gather_bitmaps(d_bm, n, world, group)
    return d_bm[: -(-n // 64)]
