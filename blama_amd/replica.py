"""Data-parallel decode replicas on one node ("replicas only").

Blama serves concurrent verification sessions; batch-1 decode does not shard,
so every GPU holds a full replica and runs its own sessions.  What is shared is
the load: rank 0 parses the GGUF and repacks the weights into its device arena
(engine.cpp Model::load), every other rank allocates an identical arena from
the GGUF header alone (mi_model_params.no_upload) and receives the bytes with
one RCCL broadcast over xGMI (torch.distributed "nccl" == RCCL on ROCm) --
a device-to-device copy instead of N host->device uploads and N repacks.

The arena is exposed to torch through __cuda_array_interface__ (no copy); the
broadcast is chunked so no single collective exceeds ``chunk_bytes``.
"""
from __future__ import annotations

from . import engine

DEFAULT_CHUNK = 1 << 30   # 1 GiB per collective


class _DeviceBytes:
    """A raw device allocation seen as a uint8 vector (CUDA array interface v3)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "strides": None, "version": 3}


def arena_tensor(model: "engine.Model", device: int):
    """The model's weight arena as a torch uint8 tensor aliasing device memory."""
    import torch
    ptr, nbytes = model.arena
    return torch.as_tensor(_DeviceBytes(ptr, nbytes), device=f"cuda:{device}")


def broadcast_bytes(t, dist, src: int = 0, chunk_bytes: int = DEFAULT_CHUNK, group=None) -> int:
    """Broadcast a flat uint8 tensor from ``src`` in chunks; returns chunks sent."""
    n = t.numel()
    k = 0
    for a in range(0, n, chunk_bytes):
        dist.broadcast(t[a:a + chunk_bytes], src=src, group=group)
        k += 1
    return k


def load_replicated(source, rank: int, local_rank: int, dist, header=None,
                    chunk_bytes: int = DEFAULT_CHUNK, group=None) -> "engine.Model":
    """Load one replica per rank.  ``source`` (path or GGUF image) must hold the
    tensor data on rank 0; other ranks only need the header (``header`` if
    given, else ``source``).  Collective: every rank of ``group`` must call it."""
    import torch
    if rank == 0:
        model = engine.Model(source, device=local_rank)
    else:
        model = engine.Model(header if header is not None else source, device=local_rank, no_upload=True)
    ptr, nbytes = model.arena
    sizes = torch.tensor([nbytes], dtype=torch.int64, device=f"cuda:{local_rank}")
    dist.all_reduce(sizes, op=dist.ReduceOp.MAX)
    if int(sizes.item()) != nbytes:
        raise engine.EngineError(f"replica arena size mismatch on rank {rank}: {nbytes} vs {int(sizes.item())}")
    torch.cuda.synchronize(local_rank)        # rank 0's repack is complete before its bytes are sent
    broadcast_bytes(arena_tensor(model, local_rank), dist, 0, chunk_bytes, group)
    torch.cuda.synchronize(local_rank)
    return model
