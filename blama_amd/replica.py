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


def _check_sizes(nbytes: int, rank: int, dist, group, device) -> None:
    """Every rank learns every rank's arena size, so a mismatch raises on ALL ranks together
    (raising only where the size differs would leave the others blocked in the broadcast)."""
    import torch
    world = dist.get_world_size(group)
    mine = torch.tensor([nbytes], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, mine, group=group)
    got = [int(x.item()) for x in sizes]
    if len(set(got)) != 1:
        raise engine.EngineError(f"replica arena sizes differ across ranks: {got} (rank {rank})")


def _src_rank(dist, group) -> int:
    """The global rank of the group's first member: the replica that parsed the GGUF."""
    return 0 if group is None else dist.get_global_rank(group, 0)


def load_replicated(source, rank: int, local_rank: int, dist, header=None,
                    chunk_bytes: int = DEFAULT_CHUNK, group=None) -> "engine.Model":
    """Load one replica per rank.  ``source`` (path or GGUF image) must hold the
    tensor data on the group's first rank; other ranks only need the header (``header`` if
    given, else ``source``).  Collective: every rank of ``group`` must call it."""
    import torch
    src = _src_rank(dist, group)
    if rank == src:
        model = engine.Model(source, device=local_rank)
    else:
        model = engine.Model(header if header is not None else source, device=local_rank, no_upload=True)
    ptr, nbytes = model.arena
    dev = "cpu" if dist.get_backend(group) == "gloo" else f"cuda:{local_rank}"
    _check_sizes(nbytes, rank, dist, group, dev)
    torch.cuda.synchronize(local_rank)        # the source's repack is complete before its bytes are sent
    broadcast_bytes(arena_tensor(model, local_rank), dist, src, chunk_bytes, group)
    torch.cuda.synchronize(local_rank)
    return model
