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
  4. each rank synthesizes its buckets on its own GPU (no collective on the data path); given
     several engines per GPU (`synth_fn` a list), consecutive buckets go to them in turn, each
     engine on a stream of its own, so one bucket's latency-bound acoustic pass runs beside
     another's MFMA-bound vocoder;
  5. gather: every rank packs its waveforms into one flat float32 buffer and sends it
     to rank 0 with an RCCL point-to-point send; its header (table and sample counts) and
     index table go over a CPU (gloo) group.  Rank 0 posts one receive per peer and handles
     the peers in the order they arrive: when a peer's header is in, its flat receive is
     posted on a stream of its own, followed on that stream by the pinned device -> host
     copy, so a peer's download starts the moment its audio lands and overlaps the other
     peers' transfers and rank 0's own last buckets; each peer is unpacked (views, original
     order) as soon as its copy completes, never behind a slower peer.

There is no all-reduce anywhere; xGMI traffic is the tokens once and the audio once.
Works with the gloo backend on CPU tensors (tests/test_dist_cpu.py).
"""
from __future__ import annotations

import contextlib
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

TAG_HDR, TAG_TABLE, TAG_FLAT = 11, 12, 13  # P2P tags of a peer's three gather messages


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
    synth_fn may be a list of such functions (engines of one GPU): bucket i runs on engine
    i mod len, on that engine's own stream (CUDA devices).
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
        # gather metadata (headers, index tables) travels on a CPU group the root can poll
        # without a device sync; under a gloo main group that is the group itself.  Every rank
        # constructs ShardedSynthesis, so the new_group call is collective.
        self.meta_group = group
        if not self.single and dist.get_backend(group) != "gloo":
            ranks = None if group is None else dist.get_process_group_ranks(group)
            self.meta_group = dist.new_group(ranks=ranks, backend="gloo")
        self._streams: Dict[int, "object"] = {}   # per peer: its receive and download (root)
        self._estreams: Dict[int, "object"] = {}  # per engine (several engines per GPU)
        self.arrivals: List[Tuple[int, str, float]] = []  # (peer, "header" | "unpacked", time): tests

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
        # ---- 4: local synthesis ----
        # The root's own audio goes to the host bucket by bucket on a side stream, overlapped with
        # the next bucket's synthesis (pinned buffers), and its lengths follow as non-blocking
        # copies read in the gather loop; the other ranks pack theirs for the gather.
        cuda = torch.device(dev).type == "cuda"
        overlap = self.rank == self.root and cuda
        side = torch.cuda.Stream(device=dev) if overlap else None
        synths = list(self.synth_fn) if isinstance(self.synth_fn, (list, tuple)) else [self.synth_fn]
        # one stream per engine when there are several (an engine orders its calls on one stream)
        estreams = [self._engine_stream(dev, k) for k in range(len(synths))] if cuda and len(synths) > 1 else None
        cur = torch.cuda.current_stream(dev) if estreams else None
        if estreams:
            for es in estreams:
                es.wait_stream(cur)  # (the broadcast tokens above)
        done = []
        for bi, bk in enumerate(mine):  # queue every bucket first: no host sync between them
            k = bi % len(synths)
            with (torch.cuda.stream(estreams[k]) if estreams else contextlib.nullcontext()):
                n_b = int(ln_h[bk].max())
                pend = None
                if n_b == 0:  # only empty utterances: nothing to synthesize, empty waveforms
                    wav = torch.zeros((len(bk), 0), dtype=torch.float32, device=dev)
                    wav_lens = np.zeros(len(bk), np.int64)
                else:
                    res = synths[k](tok_h[bk, :n_b], ln_h[bk])
                    wav, wav_lens = res[0], res[1]
                    pend = res[2] if len(res) > 2 else None
                host = lens_h = lens_ev = None
                if overlap:
                    ev = torch.cuda.Event()
                    ev.record()  # (on the current stream: the bucket's engine stream)
                    host = torch.empty(wav.shape, dtype=torch.float32, pin_memory=True)
                    with torch.cuda.stream(side):
                        side.wait_event(ev)
                        host.copy_(wav, non_blocking=True)
                    wav.record_stream(side)
                    if pend is not None or isinstance(wav_lens, torch.Tensor):
                        lv = torch.as_tensor(wav_lens, device=dev).to(torch.int64).reshape(-1)
                        if pend is not None:  # the lengths and the range word in one read
                            lv = torch.cat([lv, pend.word.to(device=dev, dtype=torch.int64).reshape(-1)])
                        lens_h = torch.empty(lv.shape, dtype=torch.int64, pin_memory=True)
                        lens_h.copy_(lv, non_blocking=True)
                        lens_ev = torch.cuda.Event()
                        lens_ev.record()
                if estreams and isinstance(wav, torch.Tensor):
                    wav.record_stream(cur)  # (allocated on the engine stream, read on this one below)
            done.append([bk, wav, wav_lens, host, pend, lens_h, lens_ev])
        if estreams:
            for es in estreams:  # what follows (packing, reruns, copies) runs on this stream
                cur.wait_stream(es)
        if self.rank == self.root:
            return self._root_gather(B, dev, done, side)
        # ---- 5 (peers): pack as [n, ids..., lens...] + flat samples, send to the root ----
        idx_list, len_list, parts = [], [], []
        for bk, wav, wav_lens, _, pend, _, _ in done:
            wav, wav_lens = self._resolve(wav, wav_lens, pend)
            for j, u in enumerate(bk):
                L = int(wav_lens[j])
                idx_list.append(u)
                len_list.append(L)
                parts.append(wav[j, :L].reshape(-1).to(device=dev, dtype=torch.float32))
        table = torch.tensor([len(idx_list)] + idx_list + len_list, dtype=torch.int64)
        flat = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.float32, device=dev)
        hdr = torch.tensor([table.numel(), flat.numel()], dtype=torch.int64)
        works = [self.dist.isend(hdr, self.root, group=self.meta_group, tag=TAG_HDR),
                 self.dist.isend(table, self.root, group=self.meta_group, tag=TAG_TABLE),
                 self.dist.isend(flat, self.root, group=self.group, tag=TAG_FLAT)]
        for w in works:
            w.wait()
        return None

    def _engine_stream(self, dev, k):
        import torch
        st = self._estreams.get(k)
        if st is None:
            st = self._estreams[k] = torch.cuda.Stream(device=dev)
        return st

    @staticmethod
    def _resolve(wav, wav_lens, pend, host_vals=None):
        """(wav, host lengths) of one bucket: reads the lengths (and the pending range word) once,
        and reruns the bucket on the fp32 encoder when the word is set (model.PendingRange)."""
        import torch
        if pend is not None:
            h = host_vals
            if h is None:
                h = torch.cat([torch.as_tensor(wav_lens, device=pend.word.device).to(torch.int64).reshape(-1),
                               pend.word.to(torch.int64).reshape(-1)]).cpu().numpy()
            return pend.resolve(wav, h[:-1], int(h[-1]))
        if host_vals is not None:
            return wav, host_vals
        if isinstance(wav_lens, torch.Tensor):
            return wav, wav_lens.cpu().numpy()
        return wav, wav_lens

    def _root_gather(self, B, dev, done, side):
        """The root's side of step 5: one receive per peer, every peer handled as it arrives.

        A thread per peer waits for that peer's header and index table on the CPU group (and,
        when the audio travels on a CPU group too, for the audio); the main thread posts each
        peer's RCCL receive + pinned download on that peer's own stream the moment its header is
        in, and unpacks whatever has landed -- the root's own buckets included -- in arrival order."""
        import queue
        import threading

        import torch
        out: List[Optional[np.ndarray]] = [None] * B
        overlap = side is not None
        peers = [r for r in range(self.world) if r != self.root]
        arrived: "queue.Queue" = queue.Queue()
        t0 = time.perf_counter()

        def meta_rx(r):
            try:
                hdr = torch.zeros(2, dtype=torch.int64)
                self.dist.irecv(hdr, r, group=self.meta_group, tag=TAG_HDR).wait()
                self.arrivals.append((r, "header", time.perf_counter() - t0))
                nt, nf = (int(v) for v in hdr.tolist())
                tab = torch.zeros(nt, dtype=torch.int64)
                self.dist.irecv(tab, r, group=self.meta_group, tag=TAG_TABLE).wait()
                flat = None
                if not overlap:  # the audio on a CPU group: received here as well
                    flat = torch.empty(nf, dtype=torch.float32)
                    self.dist.irecv(flat, r, group=self.group, tag=TAG_FLAT).wait()
                arrived.put((r, nf, tab, flat, None))
            except Exception as e:  # surfaced by the main thread
                arrived.put((r, 0, None, None, e))

        threads = [threading.Thread(target=meta_rx, args=(r,), daemon=True) for r in peers]
        for t in threads:
            t.start()
        own = list(done)
        expect = len(peers)
        landing: Dict[int, tuple] = {}
        while own or expect or landing:
            moved = False
            # the root's own buckets, in order, as their lengths reach the host
            while own and (own[0][6] is None or own[0][6].query()):
                bk, wav, wav_lens, host, pend, lens_h, _ = own.pop(0)
                wav2, wl = self._resolve(wav, wav_lens, pend, None if lens_h is None else lens_h.numpy())
                if overlap and wav2 is not wav:  # rerun on the fp32 encoder: its own copy to the host
                    host = wav2.cpu()
                for j, u in enumerate(bk):
                    L = int(wl[j])
                    out[int(u)] = host.numpy()[j, :L] if overlap else wav2[j, :L].reshape(-1).to(torch.float32).cpu().numpy()
                moved = True
            # peers whose header and table are in
            while True:
                try:
                    r, nf, tab, flat, err = arrived.get_nowait()
                except queue.Empty:
                    break
                expect -= 1
                moved = True
                if err is not None:
                    raise err
                if not overlap:
                    self._unpack(out, tab.numpy(), flat)
                    self.arrivals.append((r, "unpacked", time.perf_counter() - t0))
                    continue
                # the audio receive and its download on this peer's stream, posted at once
                st = self._streams.get(r)
                if st is None:
                    st = self._streams[r] = torch.cuda.Stream(device=dev)
                buf = torch.empty(nf, dtype=torch.float32, device=dev)
                with torch.cuda.stream(st):
                    fw = self.dist.irecv(buf, r, group=self.group, tag=TAG_FLAT)
                    fw.wait()  # (RCCL: a stream dependency, not a host wait)
                    host = torch.empty(nf, dtype=torch.float32, pin_memory=True)
                    host.copy_(buf, non_blocking=True)
                    ready = torch.cuda.Event()
                    ready.record(st)
                buf.record_stream(st)
                landing[r] = (tab, ready, host)
            # peers whose audio is on the host: unpacked at once, whatever the others do
            for r in sorted(landing):
                tab, ready, host = landing[r]
                if not ready.query():
                    continue
                self._unpack(out, tab.numpy(), host)
                self.arrivals.append((r, "unpacked", time.perf_counter() - t0))
                del landing[r]
                moved = True
            if not moved:
                time.sleep(20e-6)
        for t in threads:
            t.join()
        if overlap:
            side.synchronize()  # the root's own downloads (its views above point into them)
        return out

    @staticmethod
    def _unpack(out, t, f):
        """Views of one rank's flat audio into `out` by its [n, ids..., lens...] table."""
        if hasattr(f, "is_cuda") and f.is_cuda:
            f = torch_pinned_copy(f)
        f = f.numpy() if hasattr(f, "numpy") else f
        n = int(t[0])
        ids, ls = t[1:1 + n], t[1 + n:1 + 2 * n]
        off = 0
        for u, L in zip(ids, ls):
            out[int(u)] = f[off:off + int(L)]
            off += int(L)


def torch_pinned_copy(f):
    """One device -> host copy through a pinned buffer."""
    import torch
    return torch.empty(f.shape, dtype=f.dtype, pin_memory=True).copy_(f)
