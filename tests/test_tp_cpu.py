"""Tensor parallelism on CPU (gloo, world_size 2, 4 and 8): the rank-0-driven TP
engine (shared-memory step ring, Megatron shards, vocab-parallel embed/lm_head,
all-reduce per layer) must reproduce the single-rank model exactly in fp32,
including chunked prefill, pipelined/eager decode and session prefix reuse.  At
TP 4 and 8 tiny-llama-h8 leaves every rank one replicated kv head -- the
per-rank layout of Llama-3-70B at TP=8 (BASELINE config 4)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from omnia_amd.engine.engine import EngineConfig, LLMEngine
from omnia_amd.engine.sampling_params import SamplingParams
from omnia_amd.models.config import resolve
from omnia_amd.models.llama import LlamaModel
from omnia_amd.models.loader import shard_weights

PROMPTS = [list(range(5, 70)), list(range(100, 130)), list(range(7, 200, 3))]


def _cfg(tp, model="tiny-llama", **kw):
    kw.setdefault("use_graphs", False)
    return EngineConfig(model=model, device="cpu", dtype="float32", tp=tp, num_blocks=64,
                        block_size=32, max_batch=8, max_model_len=1024, max_prefill_tokens=64,
                        **kw)


def _generate_mixed(eng):
    """Two sequences decoding when a third prompt arrives: mixed steps."""
    p = SamplingParams(temperature=0, max_tokens=10, ignore_eos=True)
    s1 = eng.add_request(PROMPTS[0], p)
    s2 = eng.add_request(PROMPTS[1], p)
    for _ in range(4):
        eng.step()
    s3 = eng.add_request(PROMPTS[2], p)
    eng.run_until_done()
    mixed = eng.counters.get("steps_mixed", 0) + eng.counters.get("steps_mixed_sync", 0)
    return [s1.output, s2.output, s3.output], mixed


def _full_weights(model="tiny-llama"):
    from omnia_amd.models import build_model

    return build_model(resolve(model), device="cpu", dtype=torch.float32, seed=3).w


def _generate(eng):
    p = SamplingParams(temperature=0, max_tokens=12, ignore_eos=True)
    out = [s.output for s in eng.generate(PROMPTS, p, session_ids=["a", "b", "c"])]
    # second turn of session "a": prefix reuse on every rank's KV shard
    t2 = eng.generate([PROMPTS[0] + out[0] + [9, 8, 7]], p, session_ids=["a"])[0]
    return out + [t2.output], t2.prefix_hit


def _worker(rank, world, port, q, model="tiny-llama", mixed=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from omnia_amd.engine import tp
    from omnia_amd.parallel import state as pstate

    try:
        cfg = _cfg(world, model, mixed_budget=mixed, tp_mixed=bool(mixed))
        full = _full_weights(model)  # built before the TP state exists: the whole model
        pstate.init_distributed(tp_size=world, backend="gloo", device="cpu")
        w = shard_weights(full, resolve(model), world, rank)
        eng = tp.start(cfg, weights=w)
        if eng is not None:
            res = _generate_mixed(eng) if mixed else _generate(eng)
            eng.shutdown()
            q.put(("ok", res))
    except Exception as e:  # pragma: no cover - surfaced through the queue
        import traceback

        q.put(("err", traceback.format_exc()))
        raise


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_tp2_engine_matches_single_rank(model):
    """tiny-mixtral at TP=2 is expert parallel: 2 of 4 experts per rank."""
    ref = _generate(LLMEngine(_cfg(1, model), weights=_full_weights(model)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, model)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        status, res = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert status == "ok", res
    outs, hit = res
    assert hit > 0
    assert outs == ref[0]


@pytest.mark.parametrize("world", [4, 8])
def test_tp_world4_world8_engine_matches_single_rank(world):
    model = "tiny-llama-h8"
    ref = _generate(LLMEngine(_cfg(1, model), weights=_full_weights(model)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, model)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        status, res = q.get(timeout=600)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert status == "ok", res
    outs, hit = res
    assert hit > 0
    assert outs == ref[0]


def test_tp2_mixed_steps_match_single_rank():
    """Mixed prefill+decode steps under TP: rank 0 publishes each mixed step's
    packed upload (MIXED) and samples from the gathered logits; tokens equal a
    single-rank engine taking the same mixed steps."""
    ref, ref_mixed = _generate_mixed(LLMEngine(_cfg(1, mixed_budget=48),
                                               weights=_full_weights()))
    assert ref_mixed >= 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, "tiny-llama", 48))
             for r in range(2)]
    for p in procs:
        p.start()
    try:
        status, res = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert status == "ok", res
    outs, mixed = res
    assert mixed >= 2 and outs == ref


def _sim_run(eng):
    p = SamplingParams(temperature=0, max_tokens=10, ignore_eos=True)
    fill = [eng.add_request(list(range(3 + i, 20 + i)), p) for i in range(4)]
    for _ in range(4):
        eng.step()
    seqs = [eng.add_request(pr, p) for pr in PROMPTS]
    eng.run_until_done()
    return [s.output for s in fill + seqs]


def _sim_worker(rank, world, port, q, mixed):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), OMNIA_SIM_GRAPHS="1")
    try:
        from omnia_amd.engine import tp
        from omnia_amd.parallel import state as pstate
        w = shard_weights(_full_weights(), resolve("tiny-llama"), world, rank)
        pstate.init_distributed(tp_size=world, backend="gloo", device="cpu")
        eng = tp.start(_cfg(world, use_graphs=True, pipeline=True, mixed_budget=mixed,
                            tp_mixed=bool(mixed)), weights=w)
        if eng is None:
            return
        assert eng.runner.use_graphs and eng.runner.sim
        outs = _sim_run(eng)
        q.put(("ok", (outs, dict(eng.counters), eng.runner.stats.get("graph_replays", 0))))
        eng.shutdown()
    except Exception:
        import traceback
        q.put(("err", traceback.format_exc()))


@pytest.mark.parametrize("mixed", [0, 48])
def test_tp2_pipelined_graph_loop_simulated(mixed):
    """The pipelined decode loop (device token slots, placeholders, speculative
    step, graph buckets) on the CPU via OMNIA_SIM_GRAPHS, under TP=2 with
    prompts arriving while four sequences decode -- with separate and with
    mixed steps: tokens equal a synchronous single-rank engine."""
    ref = _sim_run(LLMEngine(_cfg(1, use_graphs=False, pipeline=False, mixed_budget=mixed),
                             weights=_full_weights()))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sim_worker, args=(r, 2, port, q, mixed)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        status, res = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert status == "ok", res
    outs, counters, replays = res
    assert replays > 0 and outs == ref
    if mixed:
        assert counters.get("steps_mixed", 0) >= 2


def test_shm_ring_flow_control(tmp_path):
    """The step ring: ordered delivery to every reader, payload bytes intact,
    and a full ring blocks the writer until the slowest reader releases."""
    import threading

    import numpy as np

    from omnia_amd.engine.tp import ShmRing

    path = str(tmp_path / "ring")
    w = ShmRing(path, True, nslots=2, payload=64, readers=2)
    r = ShmRing(path, False)
    got = {0: [], 1: []}

    def reader(k):
        for _ in range(5):
            h, body = r.get(k)
            got[k].append((h[0], bytes(body)))
            r.done(k)

    ts = [threading.Thread(target=reader, args=(k,)) for k in (0, 1)]
    for t in ts:
        t.start()
    for i in range(5):
        w.put([i, 7], np.arange(i + 1, dtype=np.uint8))
    for t in ts:
        t.join(10)
    want = [(i, bytes(range(i + 1))) for i in range(5)]
    assert got[0] == want and got[1] == want
    with pytest.raises(ValueError, match="exceeds"):
        w.put([9], np.zeros(65, dtype=np.uint8))
    w.put([1])
    w.put([2])  # ring of 2 now full (nobody consumes)
    with pytest.raises(TimeoutError):
        w.put([3], timeout_s=0.05)
    r.close()
    w.close(unlink=True)


def test_shm_ring_detects_dead_peers(tmp_path):
    """A reader blocked on a ring whose writer died raises within about a second
    (instead of spinning forever); so does a writer blocked on a dead reader."""
    import subprocess
    import sys

    import numpy as np

    from omnia_amd.engine.tp import ShmRing

    path = str(tmp_path / "ring")
    w = ShmRing(path, True, nslots=1, payload=8, readers=1)
    dead = subprocess.Popen([sys.executable, "-c", "pass"])
    dead.wait()
    w.ctrl[ShmRing.WRITER_PID] = dead.pid  # the writer "died"
    r = ShmRing(path, False, reader=0)
    with pytest.raises(RuntimeError, match="died"):
        r.get(0)
    with pytest.raises(TimeoutError):  # deadline, writer alive
        w.ctrl[ShmRing.WRITER_PID] = 0
        r.get(0, timeout_s=1.5)
    w.put([1], np.zeros(1, dtype=np.uint8))
    w.ctrl[ShmRing.READER_PIDS] = dead.pid  # the reader "died" holding the only slot
    with pytest.raises(RuntimeError, match="reader 0"):
        w.put([2])
    r.close()
    w.close(unlink=True)
