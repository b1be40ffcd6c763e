"""Replica path on CPU (gloo, world_size 2): chunked arena broadcast and the
header-only GGUF a non-zero rank loads from (replicas only)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from blama_amd import engine, replica, synthetic


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bcast_worker(rank, world, port, n, chunk, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.arange(n, dtype=torch.int64).to(torch.uint8) if rank == 0 else torch.zeros(n, dtype=torch.uint8)
    k = replica.broadcast_bytes(t, dist, src=0, chunk_bytes=chunk)
    ok = bool(torch.equal(t, torch.arange(n, dtype=torch.int64).to(torch.uint8)))
    q.put((rank, k, ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("n,chunk", [(10_000, 3_000), (4096, 1 << 30), (1, 7)])
def test_broadcast_bytes_gloo_ws2(n, chunk):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bcast_worker, args=(r, 2, port, n, chunk, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = (n + chunk - 1) // chunk
    assert res == [(0, want, True), (1, want, True)]


@pytest.mark.parametrize("name", ["tiny-q4_k_m", "tiny-moe-q5_k_m", "llama2-7b-q4_k_m"])
def test_header_only_image_describes_the_same_model(name):
    cfg = synthetic.CONFIGS[name]
    hdr = synthetic.build_gguf(cfg, seed=0, header_only=True)
    m = engine.Model(hdr, vocab_only=True)
    assert (m.n_vocab, m.n_embd, m.n_layer, m.n_head, m.n_head_kv) == \
        (cfg.n_vocab, cfg.n_embd, cfg.n_layer, cfg.n_head, cfg.n_head_kv)
    if cfg.n_layer <= 4:   # the full image starts with exactly these bytes
        full = synthetic.build_gguf(cfg, seed=0)
        assert np.array_equal(full[:hdr.size], hdr)


def test_device_bytes_interface():
    d = replica._DeviceBytes(0x1000, 77)
    cai = d.__cuda_array_interface__
    assert cai["shape"] == (77,) and cai["typestr"] == "|u1" and cai["data"] == (0x1000, False)


def _sizes_worker(rank, world, port, sizes, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        replica._check_sizes(sizes[rank], rank, dist, None, "cpu")
        q.put((rank, "ok"))
    except engine.EngineError as e:
        q.put((rank, "raised" if "differ" in str(e) else str(e)))
    dist.destroy_process_group()


@pytest.mark.parametrize("sizes,want", [((100, 100), "ok"), ((100, 120), "raised"), ((120, 100), "raised")])
def test_arena_size_check_raises_on_every_rank(sizes, want):
    """A mismatch must raise on ALL ranks (raising only on the smaller ranks left the
    others blocked in the broadcast)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_sizes_worker, args=(r, 2, port, sizes, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == [(0, want), (1, want)]


def _src_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = dist.new_group([1, 2])
    if rank in (1, 2):
        t = torch.full((5,), rank, dtype=torch.uint8)
        replica.broadcast_bytes(t, dist, src=replica._src_rank(dist, g), chunk_bytes=2, group=g)
        q.put((rank, replica._src_rank(dist, g), int(t[0])))
    dist.destroy_process_group()


def test_subgroup_source_is_its_first_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_src_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    assert res == [(1, 1, 1), (2, 1, 1)]


def _replica_worker(rank, world, port, q):
    """On ONE GPU: rank 0 loads the full image, rank 1 only the header (no_upload), the arena
    is broadcast over gloo, and both replicas then decode the same logits bit for bit."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = synthetic.CONFIGS["tiny-q4_k_m"]
    if rank == 0:
        m = replica.load_replicated(synthetic.build_gguf(cfg, seed=7), rank, 0, dist, chunk_bytes=1 << 20)
    else:
        m = replica.load_replicated(None, rank, 0, dist, header=synthetic.build_gguf(cfg, seed=7, header_only=True),
                                    chunk_bytes=1 << 20)
    ctx = engine.Context(m, n_ctx=32)
    ctx.decode([1, 2, 3, 4, 5])
    q.put((rank, ctx.logits().tobytes()))
    ctx.close()
    m.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_load_replicated_two_ranks_one_gpu(gpu_lib):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_replica_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=110) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
