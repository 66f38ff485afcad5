"""Multi-process CPU tests (gloo, world size 2, 3, 4 and 8) of the utterance-sharding
bookkeeping: plan, token broadcast, packed P2P gather, original order restored."""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gonova_tts_amd.dist import ShardedSynthesis, plan_buckets


def fake_synth(tokens, lens):
    """Deterministic stand-in for the GPU engine: 3 samples per token, value = token id + position."""
    B, N = tokens.shape
    wav = torch.zeros((B, 3 * N), dtype=torch.float32)
    for i in range(B):
        L = int(lens[i])
        v = np.repeat(tokens[i, :L].astype(np.float32), 3) + np.arange(3 * L, dtype=np.float32) * 1e-3
        wav[i, :3 * L] = torch.from_numpy(v)
    return wav, np.asarray(lens, np.int64) * 3


def expected(tokens, lens):
    return [fake_synth(tokens[i:i + 1, :lens[i]], lens[i:i + 1])[0][0, :3 * lens[i]].numpy() for i in range(len(lens))]


def make_batch(B=70, seed=0):
    rng = np.random.default_rng(seed)
    lens = rng.integers(29, 145, size=B).astype(np.int32)
    tok = np.zeros((B, lens.max()), np.int32)
    for i, L in enumerate(lens):
        tok[i, :L] = rng.integers(1, 78, size=L)
    return tok, lens


def make_batch_with_empties(B=40, seed=4):
    """Mixed lengths plus enough zero-length utterances that whole buckets are empty."""
    tok, lens = make_batch(B, seed)
    lens[::2] = 0
    tok[::2] = 0
    return tok, lens


def _worker(rank, world, port, q, empties=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tok, lens = make_batch_with_empties() if empties else make_batch()
        sh = ShardedSynthesis(fake_synth, torch.device("cpu"), bucket=16)
        out = sh.run(tok if rank == 0 else None, lens if rank == 0 else None)
        if rank == 0:
            exp = expected(tok, lens)
            ok = all(o is not None and np.array_equal(o, e) for o, e in zip(out, exp))
            q.put(ok)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,empties", [(2, False), (3, False), (2, True), (8, False)])  # 8: the driver's N=8 layout
def test_sharded_gather_restores_order(world, empties):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, empties)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def _slow_worker(rank, world, port, q, slow_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tok, lens = make_batch()

        def synth(t, l):
            if rank == slow_rank:
                time.sleep(1.5)
            return fake_synth(t, l)

        sh = ShardedSynthesis(synth, torch.device("cpu"), bucket=16)
        out = sh.run(tok if rank == 0 else None, lens if rank == 0 else None)
        if rank == 0:
            ok = all(o is not None and np.array_equal(o, e) for o, e in zip(out, expected(tok, lens)))
            q.put((ok, sh.arrivals))
    finally:
        dist.destroy_process_group()


def test_gather_unpacks_each_peer_as_it_arrives():
    """the root receives every peer on its own and unpacks a peer as soon as
    its audio is in -- a slow last peer (1.5 s late) does not hold the earlier peers back."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 4
    procs = [ctx.Process(target=_slow_worker, args=(r, world, port, q, world - 1)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ok, arrivals = q.get(timeout=10)
    assert ok
    t = {(r, what): at for r, what, at in arrivals}
    assert set(t) == {(r, w) for r in (1, 2, 3) for w in ("header", "unpacked")}
    for r in (1, 2):
        assert t[(r, "unpacked")] < t[(3, "header")] - 0.5, arrivals


def test_plan_is_balanced_and_complete():
    rng = np.random.default_rng(1)
    lens = rng.integers(29, 145, size=256)
    plan = plan_buckets(lens, 8, 32)
    flat = sorted(u for r in plan for bk in r for u in bk)
    assert flat == list(range(256))
    loads = [sum(int(lens[u]) for bk in r for u in bk) for r in plan]
    assert max(loads) <= 1.02 * (sum(loads) / 8)
    assert all(len(bk) <= 32 for r in plan for bk in r)


def test_plan_single_rank_keeps_everything():
    plan = plan_buckets([5, 9, 1], 1, 2)
    assert plan == [[[1, 0], [2]]]
    assert plan_buckets([], 2, 32) == [[], []]


def test_single_process_without_group():
    assert not dist.is_initialized()
    tok, lens = make_batch(B=40, seed=3)
    out = ShardedSynthesis(fake_synth, torch.device("cpu"), bucket=16).run(tok, lens)
    for o, e in zip(out, expected(tok, lens)):
        np.testing.assert_array_equal(o, e)


def test_several_engines_take_buckets_in_turn():
    """synth_fn as a list (several engines on one GPU): bucket i goes to engine i mod n, and the
    gathered result is the one-engine result, at world size 1 and under gloo at world size 2."""
    tok, lens = make_batch(B=70, seed=5)
    calls = []

    def eng(k):
        def fn(t, l):
            calls.append(k)
            return fake_synth(t, l)
        return fn

    out = ShardedSynthesis([eng(0), eng(1)], torch.device("cpu"), bucket=16).run(tok, lens)
    assert calls == [0, 1, 0, 1, 0]  # 70 utterances: 5 buckets of <= 16
    for o, e in zip(out, expected(tok, lens)):
        np.testing.assert_array_equal(o, e)


def test_all_empty_buckets_yield_empty_waveforms():
    """Zero-length utterances collect in the last buckets (longest first); a bucket made only
    of them is not sent to the engine (which rejects N = 0) and comes back as empty audio."""
    calls = []

    def synth(t, l):
        assert t.shape[1] > 0
        calls.append(len(l))
        return fake_synth(t, l)

    tok, lens = make_batch_with_empties()
    out = ShardedSynthesis(synth, torch.device("cpu"), bucket=8).run(tok, lens)
    for o, e, L in zip(out, expected(tok, lens), lens):
        assert o.shape[0] == 3 * L
        np.testing.assert_array_equal(o, e)
    assert sum(calls) < len(lens)  # the all-empty buckets never reached the engine
    out0 = ShardedSynthesis(synth, torch.device("cpu"), bucket=8).run(np.zeros((3, 4), np.int32),
                                                                      np.zeros(3, np.int32))
    assert all(o.shape == (0,) for o in out0)


class FakePending:
    """Stand-in for model.PendingRange: an unread range word; resolve() reruns the bucket."""

    def __init__(self, tokens, lens, tripped, log):
        self.word = torch.tensor([1 if tripped else 0], dtype=torch.int32)
        self.tokens, self.lens, self.log = tokens, lens, log

    def resolve(self, wav, lens_host, word_host):
        if not word_host:
            return wav, lens_host
        self.log.append(len(self.lens))
        w, wl = fake_synth(self.tokens, self.lens)
        return w, wl


def guarded_synth(log, trip_token=99):
    """host_lens=False-style engine: device-style lengths plus a pending range word; a bucket
    holding token `trip_token` "overflows": its queued audio is inf and the word is set."""
    def synth(t, l):
        wav, wl = fake_synth(t, l)
        tripped = bool((t == trip_token).any())
        if tripped:
            wav = torch.full_like(wav, float("inf"))
        return wav, torch.from_numpy(wl), FakePending(t, l, tripped, log)
    return synth


def test_range_word_read_with_lengths_and_tripped_bucket_rerun():
    """ShardedSynthesis reads a bucket's pending range word with its lengths (one host read) and
    resolves a set word by synthesizing the bucket again (model.PendingRange.resolve): no inf
    reaches the caller, the other buckets are untouched."""
    tok, lens = make_batch(B=40, seed=3)
    tok[5, 0] = 99
    log = []
    out = ShardedSynthesis(guarded_synth(log), torch.device("cpu"), bucket=8).run(tok, lens)
    assert log == [8]  # exactly the one bucket holding utterance 5 was rerun
    for o, e in zip(out, expected(tok, lens)):
        assert np.isfinite(o).all()
        np.testing.assert_array_equal(o, e)


def _guard_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tok, lens = make_batch()
        tok[:, 0] = np.where(np.arange(len(lens)) % 7 == 0, 99, tok[:, 0])
        log = []
        out = ShardedSynthesis(guarded_synth(log), torch.device("cpu"), bucket=16).run(
            tok if rank == 0 else None, lens if rank == 0 else None)
        q.put(("reran", rank, len(log)))
        if rank == 0:
            exp = expected(tok, lens)
            q.put(("ok", all(o is not None and np.isfinite(o).all() and np.array_equal(o, e) for o, e in zip(out, exp))))
    finally:
        dist.destroy_process_group()


def test_range_guard_rerun_on_every_rank_gloo():
    """The same on two gloo ranks: each rank resolves its own tripped buckets before the gather."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_guard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    msgs = [q.get(timeout=10) for _ in range(3)]
    assert ("ok", True) in msgs
    assert all(m[2] > 0 for m in msgs if m[0] == "reran")  # both ranks had a bucket to rerun
