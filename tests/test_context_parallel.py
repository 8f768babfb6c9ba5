"""Context-parallel ring-attention prefill on CPU with gloo:
zig-zag sharding round-trips, and W-rank ring attention (GQA, causal and not)
reproduces dense fp32 attention over the whole sequence at W = 2 and 4."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from omnia_amd.parallel import context_parallel as cp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_zigzag_roundtrip_and_balance():
    x = torch.arange(32).view(32, 1)
    parts = [cp.shard(x, 4, r) for r in range(4)]
    assert torch.equal(cp.unshard(parts), x)
    # causal work per rank (sum of visible keys) is equal under zig-zag
    work = [int((cp.zigzag_indices(32, 4, r) + 1).sum()) for r in range(4)]
    assert len(set(work)) == 1
    with pytest.raises(ValueError):
        cp.zigzag_indices(30, 4, 0)


def _worker(rank, world, port, causal, q_out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        T, Hq, Hkv, D = 64, 8, 2, 16
        q = torch.randn(T, Hq, D)
        k = torch.randn(T, Hkv, D)
        v = torch.randn(T, Hkv, D)
        o = cp.ring_attention(cp.shard(q, world, rank), cp.shard(k, world, rank),
                              cp.shard(v, world, rank), T, causal=causal, q_tile=5)
        parts = [torch.empty_like(o) for _ in range(world)]
        dist.all_gather(parts, o)
        if rank == 0:
            full = cp.unshard(parts)
            ref = cp.reference_attention(q, k, v, causal=causal)
            q_out.put(float((full - ref).abs().max()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,causal", [(2, True), (4, True), (2, False)])
def test_ring_attention_matches_dense(world, causal):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, causal, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    err = q.get(timeout=5)
    assert err < 1e-4, err


@pytest.mark.gpu
def test_block_merge_on_gpu_bf16():
    """The per-block product + LSE merge on the MI355X (bf16 operands through
    hipBLASLt, fp32 statistics) against dense fp32 attention."""
    torch.manual_seed(1)
    T, Hq, Hkv, D = 1024, 32, 8, 128
    dev = "cuda"
    q = torch.randn(T, Hq, D, device=dev, dtype=torch.bfloat16)
    k = torch.randn(T, Hkv, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(T, Hkv, D, device=dev, dtype=torch.bfloat16)
    pos = torch.arange(T, device=dev)
    scale = D ** -0.5
    h = T // 2
    o1, l1 = cp._block(q, k[:h], v[:h], pos, pos[:h], scale, True, 256)
    o2, l2 = cp._block(q, k[h:], v[h:], pos, pos[h:], scale, True, 256)
    o, _ = cp._merge(o1, l1, o2, l2)
    ref = cp.reference_attention(q.float(), k.float(), v.float(), scale=scale)
    assert (o - ref).abs().max().item() < 3e-2
