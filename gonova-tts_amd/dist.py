"""Utterance sharding across the GPUs of one node.

The reference has no parallelism: it scales out by running one server process per GPU
(`server.py:397-400,486-488`) behind an external load balancer.  Here one process per
GPU (torch.distributed, backend "nccl" = RCCL over xGMI) shares one request batch:

  1. rank 0 owns the batch: token matrix int32 [B, N] + lengths [B];
  2. one broadcast of [B, N] + [B] (~147 KB at B=256, N=144) -- the "scatter": every
     rank derives the same deterministic plan and keeps only its rows;
  3. plan: deal utterances longest-first to the least-loaded rank (longest processing
     time first, load = total tokens, at most ceil(B / world) utterances per rank), then
     each rank cuts its share, sorted by length, into buckets of `bucket` utterances (one
     engine call each);
  4. each rank synthesizes its buckets on its own GPU (no collective on the data path);
  5. gather: every rank packs its waveforms into one flat float32 buffer and sends it
     to rank 0 with RCCL point-to-point (batch_isend_irecv -> ncclSend/ncclRecv in one
     group); rank 0 restores the original order.

There is no all-reduce anywhere; xGMI traffic is the tokens once and the audio once.
Works with the gloo backend on CPU tensors (tests/test_dist_cpu.py).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np


def plan_buckets(lengths: Sequence[int], world: int, bucket: int = 32) -> List[List[List[int]]]:
    """-> per rank, a list of buckets (lists of utterance indices). Deterministic.

    Utterances are dealt longest-first to the least-loaded rank (load = total tokens,
    each rank capped at ceil(B / world) utterances), then each rank cuts its share,
    sorted by length, into buckets of <= `bucket`.  Balancing at utterance
    granularity is possible because the engine runs ragged batches natively (rows
    past an utterance's length exit early), so mixing lengths inside a bucket costs
    little while bucket-granular assignment would leave ranks idle."""
    lengths = np.asarray(lengths, np.int64)
    B = len(lengths)
    cap = -(-B // world) if B else 0
    order = np.argsort(-lengths, kind="stable")
    load = np.zeros(world, np.int64)
    count = np.zeros(world, np.int64)
    share: List[List[int]] = [[] for _ in range(world)]
    for u in order:
        cand = [r for r in range(world) if count[r] < cap]
        r = min(cand, key=lambda q: (load[q], q))
        share[r].append(int(u))
        load[r] += int(lengths[u])
        count[r] += 1
    plan: List[List[List[int]]] = []
    for r in range(world):
        s = sorted(share[r], key=lambda u: (-int(lengths[u]), u))
        plan.append([s[i:i + bucket] for i in range(0, len(s), bucket)])
    return plan


SynthFn = Callable[[np.ndarray, np.ndarray], Tuple["object", np.ndarray]]


class ShardedSynthesis:
    """Run one batch of utterances across all ranks of a process group, results on `root`.

    synth_fn(tokens int32 [b, N], lens int32 [b]) -> (wav tensor [b, S] float32, wav_lens int64 [b])
    or (wav, wav_lens, pending) runs on the calling rank's device (a GonovaTTS.synthesize_tokens, or
    a fake on CPU).  wav_lens may be a numpy array or a device tensor; with device tensors
    (synthesize_tokens(..., host_lens=False)) every bucket is queued before the first host sync.
    `pending` (model.PendingRange, or None) carries the bucket's unread range word: it is read in
    the same device -> host copy as the lengths, and a bucket whose word is set is synthesized
    again on the fp32 encoder there (pending.resolve) before its audio is packed.  On the root the
    waveforms come back as views into one host buffer per rank (one pinned D2H copy each).
    """

    def __init__(self, synth_fn: SynthFn, device, group=None, root: int = 0, bucket: int = 32):
        import torch.distributed as dist
        self.dist = dist
        self.synth_fn = synth_fn
        self.device = device
        self.group = group
        self.root = root
        self.bucket = bucket
        self.single = not dist.is_initialized()  # one process, no group: same code path, no comms
        self.rank = 0 if self.single else dist.get_rank(group)
        self.world = 1 if self.single else dist.get_world_size(group)
        if self.single:
            self.root = 0

    def _bcast(self, t):
        if not self.single:
            self.dist.broadcast(t, src=self.root, group=self.group)
        return t

    def run(self, tokens: Optional[np.ndarray] = None, lens: Optional[np.ndarray] = None):
        import torch
        dev = self.device
        # ---- 1-2: broadcast the batch (shape first) ----
        meta = torch.zeros(2, dtype=torch.int64, device=dev)
        if self.rank == self.root:
            meta[0], meta[1] = int(tokens.shape[0]), int(tokens.shape[1])
        self._bcast(meta)
        B, N = int(meta[0]), int(meta[1])
        tok = torch.zeros((B, N), dtype=torch.int32, device=dev)
        ln = torch.zeros((B,), dtype=torch.int32, device=dev)
        if self.rank == self.root:
            tok.copy_(torch.from_numpy(np.ascontiguousarray(tokens, np.int32)))
            ln.copy_(torch.from_numpy(np.ascontiguousarray(lens, np.int32)))
        self._bcast(tok)
        self._bcast(ln)
        tok_h, ln_h = tok.cpu().numpy(), ln.cpu().numpy()
        # ---- 3: deterministic plan ----
        plan = plan_buckets(ln_h, self.world, self.bucket)
        mine = plan[self.rank]
        # ---- 4: local synthesis, packed as [index, length] table + flat samples ----
        idx_list, len_list, parts = [], [], []
        done = []
        # the root's own audio goes to the host bucket by bucket on a side stream, overlapped
        # with the next bucket's synthesis (pinned, cached buffers); the other ranks pack theirs
        # for the gather
        overlap = self.rank == self.root and torch.device(dev).type == "cuda"
        side = torch.cuda.Stream(device=dev) if overlap else None
        for bk in mine:  # queue every bucket first: no host sync between them
            n_b = int(ln_h[bk].max())
            pend = None
            if n_b == 0:  # only empty utterances: nothing to synthesize, empty waveforms
                wav = torch.zeros((len(bk), 0), dtype=torch.float32, device=dev)
                wav_lens = np.zeros(len(bk), np.int64)
            else:
                res = self.synth_fn(tok_h[bk, :n_b], ln_h[bk])
                wav, wav_lens = res[0], res[1]
                pend = res[2] if len(res) > 2 else None
            host = None
            if overlap:
                ev = torch.cuda.Event()
                ev.record()
                host = torch.empty(wav.shape, dtype=torch.float32, pin_memory=True)
                with torch.cuda.stream(side):
                    side.wait_event(ev)
                    host.copy_(wav, non_blocking=True)
                wav.record_stream(side)
            done.append((bk, wav, wav_lens, host, pend))
        own = []
        for bk, wav, wav_lens, host, pend in done:
            if pend is not None:  # the lengths and the range word in one read
                h = torch.cat([torch.as_tensor(wav_lens, device=pend.word.device).to(torch.int64).reshape(-1),
                               pend.word.to(torch.int64).reshape(-1)]).cpu().numpy()
                wav2, wav_lens = pend.resolve(wav, h[:-1], int(h[-1]))
                if wav2 is not wav:  # rerun on the fp32 encoder: its own copy to the host
                    wav = wav2
                    if overlap:
                        host = wav.cpu()
            elif isinstance(wav_lens, torch.Tensor):
                wav_lens = wav_lens.cpu().numpy()
            if overlap:
                own.append((bk, wav_lens, host))
                continue
            for j, u in enumerate(bk):
                L = int(wav_lens[j])
                idx_list.append(u)
                len_list.append(L)
                parts.append(wav[j, :L].reshape(-1).to(device=dev, dtype=torch.float32))
        table = torch.tensor([len(idx_list)] + idx_list + len_list, dtype=torch.int64, device=dev)
        flat = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.float32, device=dev)
        # ---- 5: gather to root (sizes first, then one P2P group) ----
        sizes = torch.tensor([table.numel(), flat.numel()], dtype=torch.int64, device=dev)
        all_sizes = [torch.zeros_like(sizes) for _ in range(self.world)]
        if self.single:
            all_sizes[0] = sizes
        else:
            self.dist.all_gather(all_sizes, sizes, group=self.group)
        if self.rank != self.root:
            ops = [self.dist.P2POp(self.dist.isend, table, self.root, self.group),
                   self.dist.P2POp(self.dist.isend, flat, self.root, self.group)]
            for r in self.dist.batch_isend_irecv(ops):
                r.wait()
            return None
        tables, flats, ops = {}, {}, []
        for r in range(self.world):
            if r == self.root:
                continue
            nt, nf = int(all_sizes[r][0]), int(all_sizes[r][1])
            tables[r] = torch.zeros(nt, dtype=torch.int64, device=dev)
            flats[r] = torch.zeros(nf, dtype=torch.float32, device=dev)
            ops.append(self.dist.P2POp(self.dist.irecv, tables[r], r, self.group))
            ops.append(self.dist.P2POp(self.dist.irecv, flats[r], r, self.group))
        if ops:
            for q in self.dist.batch_isend_irecv(ops):
                q.wait()
        tables[self.root], flats[self.root] = table, flat
        out: List[Optional[np.ndarray]] = [None] * B
        if overlap:
            side.synchronize()
            for bk, wav_lens, host in own:
                h = host.numpy()
                for j, u in enumerate(bk):
                    out[int(u)] = h[j, :int(wav_lens[j])]
        for r in range(self.world):
            if overlap and r == self.root:
                continue
            t = tables[r].cpu().numpy()
            f = flats[r]
            if f.is_cuda:  # one D2H copy through a pinned (cached) host buffer
                f = torch.empty(f.shape, dtype=f.dtype, pin_memory=True).copy_(f)
            f = f.numpy()
            n = int(t[0])
            ids, ls = t[1:1 + n], t[1 + n:1 + 2 * n]
            off = 0
            for u, L in zip(ids, ls):
                out[int(u)] = f[off:off + int(L)]
                off += int(L)
        return out
