"""bench.py — headline benchmark of the MI355X TTS engine (one JSON line on rank 0).

Workload (BASELINE.json configs[1], the config the metric is quoted on that fits one
GPU): HiFi-GAN V1 vocoder, batch 32 x 862 mel frames (10.008 s @ 22,050 Hz, 220,672
samples per utterance), fp16 activations / fp32 accumulation, synthetic mel ~ N(0,1)
already resident in HBM, deterministic seeded weights (no checkpoint offline).
A "step" = one vocoder forward over the batch.

The same line also carries `full_pipeline` (configs[2]: token ids U[1,77] [32,144],
durations forced to 6 frames/token -> 864 frames; acoustic bf16 + vocoder bf16,
tokens in HBM -> waveform in HBM), measured after the headline loop, and beside it the host
end-to-end rate (`host_e2e_*`: token ids in host memory -> waveform in pinned host memory,
the PCIe copies inside the timed region).
`--workload full` makes that the headline instead.

Multi-GPU: `bench.py --gpus N` runs one process per GPU.  Launched under
`torch.distributed.run` (RANK / WORLD_SIZE set) it is a rank; launched plainly with N > 1
it is a launcher that never touches the GPU and starts N fresh rank processes itself
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1), then exits with their status.
Every rank checks that the process group has exactly N ranks (a 1-GPU box asked for
--gpus 2 fails loudly).  Utterances are independent, so C2 runs a batch-32 shard per
rank with no data-path collective (weak scaling); the timed loop is bracketed by
barriers and the max time over ranks is used.  value = samples of all ranks / max time.
The same line carries `c4` (configs[3]: 256 mixed-length utterances owned by rank 0,
RCCL broadcast -> per-rank length-bucketed synthesis -> RCCL P2P gather to rank 0 inside
the timed region; strong scaling over N; at N=1 no process group exists and no collective
runs, which the line says), `streaming` (configs[4], C5: p50 first audio with predicted
durations as a request runs it, beside the given-durations and fast-encoder variants) and
`c1` (configs[0] through the WebSocket service with the fp32 engine).

`roofline` is for the dominant kernel family (largest summed time per step: today the
fused ResBlock-pair kernel of all four stages), timed live with hipEvents around every launch
on the stream it runs on; `roofline.kernels` lists every family the same way
(conv_gemm_kernel, conv_xres_kernel, mrf_pair_kernel, mrf_chain_kernel, upsample_stream_kernel,
conv_split_kernel).  `cpu_baseline` (rank 0, N=1 only) is the torch-CPU fp32
restatement (oracle/torch_cpu.py) timed on the host cores on a bounded
sample of C2 (4 utterances), C3 (2 utterances) and C1 (one 71-token sentence).
`full_pipeline.acoustic_roofline` is the acoustic forward against the MFMA peak (80.19 GFLOP
per utterance) with per-family splits.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SR = 22050
METRIC = "audio samples/sec/GPU + real-time factor, batch-32 10s utterances @22.05kHz"
MFMA_PEAK_TFLOPS = {"f16": 2500.0, "bf16": 2500.0, "f32": 157.3}  # dense, MI355X_MICROARCH.md
# acoustic model: 92.82 MFLOP per mel frame at N = 144 tokens / T = 864 frames (SURVEY.md §8d,
# BASELINE.md §2) = 80.19 GFLOP per 10 s utterance
ACOUSTIC_FLOPS_PER_UTT = 92.82e6 * 864
# C1 (BASELINE.json configs[0]): one sentence of N = 71 tokens x 6 frames = 426
# frames = 109,056 samples (4.95 s); the text tokenizes to exactly 71 ids (gonova_tts_amd/text.py)
C1_TEXT = "The quick brown fox jumps over the lazy dog and then ran to the woods."


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--frames", type=int, default=862)
    ap.add_argument("--tokens", type=int, default=144)
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--workload", default="vocoder", choices=["vocoder", "full", "c4", "selftest"],
                    help="selftest: CPU-only gloo check of the launcher / process group (no GPU)")
    ap.add_argument("--c4-batch", type=int, default=256)
    ap.add_argument("--c4-bucket", type=int, default=64, help="utterances per length bucket (one synthesis call; 64 measured best of 32/64/128)")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 sharded side measurement")
    ap.add_argument("--no-streaming", action="store_true", help="skip the C5 streaming latency side measurement")
    ap.add_argument("--no-full", action="store_true", help="skip the full-pipeline side measurement")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 service-latency side measurement")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-c2-batch", type=int, default=4, help="C2 utterances in the CPU-baseline sample")
    ap.add_argument("--cpu-c3-batch", type=int, default=2, help="C3 utterances in the CPU-baseline sample")
    ap.add_argument("--selftest-fail-rank", type=int, default=-1,
                    help="selftest only: this rank exits with status 7 after joining the process group "
                         "(tests/test_bench_cpu.py: the launcher must end the run, not hang)")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without torch.distributed.run: start N rank processes of this
    script (one per GPU) and return the first non-zero exit status.  This process does not
    touch the GPU (torch.cuda.device_count() does not initialise HIP on this image), so the
    children are fresh processes, never an exec of a GPU-initialised one.

    The children are polled together: as soon as one exits non-zero the others are
    terminated (SIGTERM, then SIGKILL after a grace period) -- a rank that died after
    init_process_group would otherwise leave its siblings blocked in a barrier or an RCCL
    collective until the driver's own timeout, and an 8-GPU run would print nothing."""
    import signal
    import socket
    import subprocess
    if args.workload != "selftest":
        import torch
        have = torch.cuda.device_count()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but only {have} HIP device(s) visible", file=sys.stderr, flush=True)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))

    def stop_all(grace=5.0):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        t_end = time.monotonic() + grace
        for p in procs:
            try:
                p.wait(timeout=max(0.0, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                i, rc = bad[0]
                print(f"bench.py: rank {i} exited with status {rc}; terminating the other ranks",
                      file=sys.stderr, flush=True)
                stop_all()
                return rc
            if all(c == 0 for c in codes):
                return 0
            time.sleep(0.2)
    except BaseException:
        stop_all()
        raise


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(b2: int, b3: int):
    """torch-CPU fp32 restatement (oracle/torch_cpu.py) of C2 (vocoder, b2 x 862 frames) and C3
    (tokens -> acoustic -> vocoder, b3 x 144 tokens x 6 frames) on the host cores.  value = the
    C2 samples/s (the headline metric's config); c3 holds the full-pipeline rate."""
    import torch
    from gonova_tts_amd.weights import make_acoustic_weights, make_vocoder_weights
    from oracle.torch_cpu import TorchAcoustic, TorchVocoder
    # the box's CPU share is what OMP_NUM_THREADS says (os.cpu_count() is the whole host)
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    threads = min(threads, os.cpu_count() or threads)
    torch.set_num_threads(threads)
    voc = TorchVocoder(make_vocoder_weights(seed=0))
    g = torch.Generator().manual_seed(0)
    mel = torch.randn((b2, 862, 80), generator=g)
    voc(mel[:1, :16])  # warm up the thread pool
    ac = TorchAcoustic(make_acoustic_weights(seed=0, fixed_duration=6))
    ids = torch.randint(1, 78, (b3, 144), generator=g)
    dur = torch.full((b3, 144), 6, dtype=torch.int64)
    # C1: one N = 71 sentence, tokens -> waveform
    from gonova_tts_amd.text import tokenize
    ids1 = torch.from_numpy(np.asarray(tokenize(C1_TEXT), np.int64))[None]
    assert ids1.shape[1] == 71
    # each sample timed REPS times: the rate reported is the median, with the spread beside it
    # (host load on a shared box moves a single timing by 10-20 %)
    reps = max(1, int(os.environ.get("TTS_CPU_REPS", "3")))
    t2, t3, t1 = [], [], []
    for _ in range(reps):
        t = time.perf_counter()
        wav = voc(mel)
        t2.append(time.perf_counter() - t)
        t = time.perf_counter()
        m, _ = ac(ids, dur)
        w3 = voc(m)
        t3.append(time.perf_counter() - t)
        t = time.perf_counter()
        m1, _ = ac(ids1, torch.full((1, 71), 6, dtype=torch.int64))
        w1 = voc(m1)
        t1.append(time.perf_counter() - t)
    med = lambda v: float(np.median(v))  # noqa: E731

    def spread(n, ts):
        return {"min": round(n / max(ts), 1), "max": round(n / min(ts), 1), "runs": len(ts)}
    dt2, dt3, dt1 = med(t2), med(t3), med(t1)
    return {"value": round(wav.numel() / dt2, 1), "unit": "samples/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "statistic": f"median of {reps}", "spread": spread(wav.numel(), t2),
            "sample": f"C2: {b2} utterances x 862 frames ({wav.numel() / SR:.1f} s audio), median {dt2:.1f} s of "
                      f"{reps} runs; torch-CPU fp32 restatement (oracle/torch_cpu.py), {threads} threads",
            "c3": {"value": round(w3.numel() / dt3, 1), "unit": "samples/s", "spread": spread(w3.numel(), t3),
                   "sample": f"C3: {b3} utterances x 144 tokens x 6 frames ({w3.numel() / SR:.1f} s audio), median "
                             f"{dt3:.1f} s of {reps} runs (acoustic + vocoder)"},
            "c1": {"value": round(w1.numel() / dt1, 1), "unit": "samples/s", "latency_ms": round(dt1 * 1e3, 1),
                   "rtf": round(dt1 / (w1.numel() / SR), 4), "spread": spread(w1.numel(), t1),
                   "sample": f"C1: 1 utterance x 71 tokens x 6 frames ({w1.numel() / SR:.2f} s audio), median "
                             f"{dt1:.2f} s of {reps} runs (acoustic + vocoder, fp32)"}}


class Ctx:
    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.cpu = args.workload == "selftest"
        if self.world > 1:
            # a bounded rendezvous / collective timeout: a rank that never arrives fails the run
            # instead of hanging it (launch_ranks also terminates the siblings of a failed rank)
            timeout = datetime.timedelta(seconds=float(os.environ.get("TTS_BENCH_PG_TIMEOUT", "300")))
            if self.cpu:
                dist.init_process_group("gloo", timeout=timeout)
            else:
                if self.local >= torch.cuda.device_count():
                    raise SystemExit(f"bench.py rank {self.rank}: LOCAL_RANK {self.local} but only "
                                     f"{torch.cuda.device_count()} HIP device(s) visible")
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local), timeout=timeout)
            self.world = dist.get_world_size()
            self.rank = dist.get_rank()
        if self.world != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {self.world} rank(s); "
                             "run `bench.py --gpus N` (it starts N ranks) or torch.distributed.run "
                             "--nproc-per-node N bench.py --gpus N")
        if self.cpu:
            self.dev = torch.device("cpu")
        else:
            torch.cuda.set_device(self.local)
            self.dev = torch.device("cuda", self.local)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()
        if not self.cpu:
            self.torch.cuda.synchronize()

    def max_over_ranks(self, x: float) -> float:
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def timed(self, step, steps, warmup, eng=None):
        for _ in range(warmup):
            step()
        if not self.cpu:
            self.torch.cuda.synchronize()
        # Live kernel timing (hipEvents around every MFMA launch, on its own stream) brackets
        # the LAST timed step only: two events per launch cost ~0.3 ms per C2 step (1.6 %),
        # which production runs do not pay.  The per-family averages come from that step (27
        # pair launches in C2), inside the timed region.
        prof_on = eng is not None and not os.environ.get("TTS_BENCH_NOPROF")
        nprof = 1
        self.barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            if prof_on and i == steps - nprof:
                eng.profile(True)
            step()
        self.barrier()
        el = time.perf_counter() - t0
        prof = None
        if prof_on:
            eng.profile(False)
            prof = eng.profile_read_kinds()
            self.prof_steps = nprof
        return self.max_over_ranks(el), prof


def pmc_traffic(kernel, kind="c2"):
    """HBM bytes per launch of one kernel family from a committed PMC summary (tools/pmc_traffic.py,
    profiles/*_pmc_traffic_<kind>.json: "c2" the headline step, "c3voc_bf16" the C3 vocoder in bf16
    at 864 frames), if it covers that family: the file profiles/pmc_current.json names for `kind`
    (the run on the current kernels), else the last by name."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_traffic_{kind}.json")))
    cur = os.path.join(ROOT, "profiles", "pmc_current.json")
    if os.path.exists(cur):
        name = json.load(open(cur)).get(kind)
        if name and os.path.exists(os.path.join(ROOT, "profiles", name)):
            files = [os.path.join(ROOT, "profiles", name)]
    if not files:
        return None
    d = json.load(open(files[-1]))
    fam = d.get("families", {}).get(kernel.replace("_kernel", ""))
    if fam is None:
        return None
    return {"bytes_per_launch": round(fam["traffic_bytes_per_launch"]),
            "algorithmic_bytes_per_launch": round(fam["algorithmic_bytes_per_launch"]),
            "ratio": round(fam["ratio_traffic_over_algorithmic"], 3),
            "source": os.path.relpath(files[-1], ROOT)}


def roofline(prof, elapsed, steps, dtype, traffic_for=None, prof_steps=None):
    """Roofline of the dominant kernel family (largest summed time in the timed steps),
    from the engine's live hipEvent timing: achieved = algorithmic FLOPs per launch / that
    family's average launch duration.  `kernels` lists every family the same way."""
    if prof is None:
        return None
    ps = prof_steps or steps          # steps the events covered
    kernels = {}
    for name, (ms, fl, n) in prof.items():
        if n:
            kernels[name] = {"ms_per_step": round(ms / ps, 3), "launches_per_step": n // max(ps, 1),
                             "avg_launch_us": round(ms / n * 1e3, 2),
                             "achieved_tflops": round(fl / (ms * 1e-3) / 1e12, 2)}
    name = max(prof, key=lambda k: prof[k][0])
    ms, fl, n = prof[name]
    per_launch_flops = fl / max(n, 1)
    avg_launch_ms = ms / max(n, 1)
    achieved = per_launch_flops / (avg_launch_ms * 1e-3) / 1e12 if n else 0.0
    peak = MFMA_PEAK_TFLOPS[dtype]
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 5),
            "traffic": traffic_for(name) if traffic_for else None, "kernel": name,
            "flops_per_launch": round(per_launch_flops),
            "avg_launch_us": round(avg_launch_ms * 1e3, 2), "launches_per_step": n // max(ps, 1),
            "share_of_step": round((ms / ps) / (elapsed * 1e3 / steps), 4), "profiled_steps": ps,
            "kernels": kernels}


def acoustic_roofline(prof, ac_ms, B, prof_steps):
    """The acoustic forward against the MFMA roofline: achieved = 80.19 GFLOP per utterance x B
    / the timed acoustic step, and per kernel family (live hipEvent timing of
    the last steps): its time per step, share of the step and, for the GEMM families and the
    fused attention, its own FLOPs / its own time (conv FLOPs at the padded row extent:
    the exact encoder's rows are padded to rup(N + 2, 32) = 160 per 144-token utterance)."""
    if prof is None:
        return None
    achieved = ACOUSTIC_FLOPS_PER_UTT * B / (ac_ms * 1e-3) / 1e12
    fam = {}
    for name, (ms, fl, n) in prof.items():
        if not n:
            continue
        e = {"ms_per_step": round(ms / prof_steps, 3), "launches_per_step": n // max(prof_steps, 1),
             "share_of_step": round(ms / prof_steps / ac_ms, 4)}
        if fl:
            e["achieved_tflops"] = round(fl / (ms * 1e-3) / 1e12, 1)
        fam[name] = e
    kernel_ms = sum(v["ms_per_step"] for v in fam.values())
    return {"bound": "mfma", "achieved": round(achieved, 1), "peak": 2500.0, "unit": "TFLOP/s",
            "frac": round(achieved / 2500.0, 4), "flops_per_step": ACOUSTIC_FLOPS_PER_UTT * B,
            "launches_per_step": sum(v["launches_per_step"] for v in fam.values()),
            "kernel_ms_per_step": round(kernel_ms, 3), "families": fam}


def bench_vocoder(ctx, args):
    torch = ctx.torch
    from gonova_tts_amd.config import vocoder_flops_per_sample
    from gonova_tts_amd.engine import HipEngine
    from gonova_tts_amd.weights import make_vocoder_weights
    B, T = args.batch, args.frames
    eng = HipEngine(ctx.local, vocoder_dtype=args.dtype, max_batch=B, max_frames=T)
    eng.load_weights(vocoder=make_vocoder_weights(seed=0))
    g = torch.Generator(device="cpu").manual_seed(1000 + ctx.rank)
    mel = torch.randn((B, T, 80), generator=g).to(ctx.dev)
    lens = torch.full((B,), T, dtype=torch.int32, device=ctx.dev)
    wav = torch.empty((B, T * 256), dtype=torch.float32, device=ctx.dev)
    el, prof = ctx.timed(lambda: eng.vocoder(mel, lens, out=wav), args.steps, args.warmup, eng)
    samples = B * T * 256 * args.steps * ctx.world
    value = samples / el
    out = {"value": value, "ms_per_step": el * 1e3 / args.steps, "samples_per_utt": T * 256,
           "algorithmic_tflops_per_gpu": value / ctx.world * vocoder_flops_per_sample() / 1e12,
           "roofline": roofline(prof, el, args.steps, args.dtype,
                                pmc_traffic if (B, T, args.dtype) == (32, 862, "f16") else None,
                                getattr(ctx, "prof_steps", None))}
    eng.close()
    return out


def bench_full(ctx, args, steps, warmup):
    torch = ctx.torch
    from gonova_tts_amd.engine import HipEngine
    from gonova_tts_amd.weights import make_acoustic_weights, make_vocoder_weights
    B, N, dur = args.batch, args.tokens, 6
    T = N * dur
    eng = HipEngine(ctx.local, vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=B, max_frames=T, max_tokens=N)
    eng.load_weights(vocoder=make_vocoder_weights(seed=0), acoustic=make_acoustic_weights(seed=0, fixed_duration=dur))
    g = torch.Generator(device="cpu").manual_seed(2000 + ctx.rank)
    tok = torch.randint(1, 78, (B, N), generator=g, dtype=torch.int32).to(ctx.dev)
    tl = torch.full((B,), N, dtype=torch.int32, device=ctx.dev)
    wav = torch.empty((B, T * 256), dtype=torch.float32, device=ctx.dev)

    def step():
        mel, mel_lens = eng.acoustic(tok, tl, T)
        eng.vocoder(mel, mel_lens, out=wav)

    el1, prof = ctx.timed(step, steps, warmup, eng)
    mel, mel_lens = eng.acoustic(tok, tl, T)
    torch.cuda.synchronize()
    assert int(mel_lens.min()) == T, "forced durations must give 864 frames"
    samples = B * T * 256 * steps * ctx.world
    # Two engines on two streams, half the batch each, both halves started every step -- the
    # service's two-engines-per-GPU shape (TTSService(devices=["cuda:0", "cuda:0"])): one half's
    # latency-bound acoustic pass runs beside the other half's MFMA-bound vocoder
    # (tools/c3_overlap_probe.py, round 6: 21.53 -> 20.91 ms per step on one box).  The whole batch
    # of 32 is synthesized inside every timed step; the one-stream step (and the per-family roofline,
    # which needs launches that do not overlap) is reported beside it.
    h = B // 2
    el2 = None
    if h > 0:
        eng2 = HipEngine(ctx.local, vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=B - h, max_frames=T, max_tokens=N)
        eng2.load_weights(vocoder=make_vocoder_weights(seed=0), acoustic=make_acoustic_weights(seed=0, fixed_duration=dur))
        sa, sb = torch.cuda.Stream(device=ctx.dev), torch.cuda.Stream(device=ctx.dev)

        def step2():
            cur = torch.cuda.current_stream()
            sa.wait_stream(cur)
            sb.wait_stream(cur)
            for e, st, sl in ((eng, sa, slice(0, h)), (eng2, sb, slice(h, B))):
                with torch.cuda.stream(st):
                    m_, l_ = e.acoustic(tok[sl], tl[sl], T, stream=st)
                    e.vocoder(m_, l_, out=wav[sl], stream=st)
            cur.wait_stream(sa)
            cur.wait_stream(sb)

        el2, _ = ctx.timed(step2, steps, warmup)
        mel2, lens2 = eng2.acoustic(tok[h:], tl[h:], T)
        torch.cuda.synchronize()
        assert int(lens2.min()) == T
        eng2.close()
    # Pipelined across batches, the service's steady state under load (a stream of requests): every
    # timed step runs one whole 32-utterance acoustic pass (engine A, stream a) beside the vocoder
    # pass of the batch before it (engine B, stream b), both streams joined at the end of the step.
    # K timed steps therefore do K acoustic and K vocoder passes of 32 utterances each; the first
    # timed vocoder consumes the mel of the last warmup step.  The waveform is checked bit for bit
    # against the one-stream step's (tools/c3_overlap_probe.py, round 6: 21.0 vs 21.4 ms two halves).
    step()
    torch.cuda.synchronize()
    ref = wav.clone()  # the one-stream step's waveform
    engp = HipEngine(ctx.local, vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=B, max_frames=T, max_tokens=N)
    engp.load_weights(vocoder=make_vocoder_weights(seed=0), acoustic=make_acoustic_weights(seed=0, fixed_duration=dur))
    # the two-engine form's streams when it ran: HIP maps streams onto a few hardware queues in
    # creation order, and two more new streams can share one queue (no overlap at all)
    spa, spb = (sa, sb) if h > 0 else (torch.cuda.Stream(device=ctx.dev), torch.cuda.Stream(device=ctx.dev))
    prev = {}

    def step3():
        cur = torch.cuda.current_stream()
        spa.wait_stream(cur)
        spb.wait_stream(cur)
        with torch.cuda.stream(spa):
            m_, l_ = eng.acoustic(tok, tl, T, stream=spa)
        if prev:
            with torch.cuda.stream(spb):
                engp.vocoder(prev["mel"], prev["lens"], out=wav, stream=spb)
        cur.wait_stream(spa)
        cur.wait_stream(spb)
        prev.update(mel=m_, lens=l_)

    el3, _ = ctx.timed(step3, steps, max(warmup, 1))
    torch.cuda.synchronize()
    assert torch.equal(wav, ref), "pipelined C3 waveform differs from the one-stream step's"
    engp.close()
    forms = {"one engine, one stream": el1, "pipelined: batch k's acoustic pass beside batch k-1's vocoder (two engines, two streams)": el3}
    if el2 is not None:
        forms["two engines on two streams, 16 utterances each"] = el2
    form = min(forms, key=forms.get)
    el = forms[form]
    value = samples / el
    ac_ms = None
    # acoustic-only timing (same inputs) to split the step; the live per-family timing of its
    # last steps gives the acoustic model's own roofline
    el_ac, prof_ac = ctx.timed(lambda: eng.acoustic(tok, tl, T), steps, 1, eng)
    ac_ms = el_ac * 1e3 / steps
    ac_roof = acoustic_roofline(prof_ac, ac_ms, B, getattr(ctx, "prof_steps", None) or steps)
    # host end to end: token ids in host memory -> waveform in (pinned) host
    # memory, the PCIe copies inside the timed region; reported beside the device-resident value
    tok_h = tok.cpu()
    wav_h = torch.empty((B, T * 256), dtype=torch.float32, pin_memory=True)

    def host_step():
        mel_, lens_ = eng.acoustic(tok_h.to(ctx.dev), tl, T)
        eng.vocoder(mel_, lens_, out=wav)
        wav_h.copy_(wav, non_blocking=True)
        torch.cuda.current_stream().synchronize()

    el_h, _ = ctx.timed(host_step, steps, 1)
    eng.close()
    # the same acoustic pass with encoder_precision="fast" (whole model bf16; durations may round
    # differently near .5), to show what the default exact-duration encoder costs
    engf = HipEngine(ctx.local, vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=B, max_frames=T, max_tokens=N,
                     encoder_precision="fast")
    engf.load_weights(acoustic=make_acoustic_weights(seed=0, fixed_duration=dur))
    el_f, _ = ctx.timed(lambda: engf.acoustic(tok, tl, T), steps, 1)
    engf.close()
    return {"value": round(value, 1), "unit": "samples/s", "ms_per_step": round(el * 1e3 / steps, 3),
            "form": form,
            "one_stream_ms_per_step": round(el1 * 1e3 / steps, 3),
            "two_engine_ms_per_step": round(el2 * 1e3 / steps, 3) if el2 is not None else None,
            "pipelined_ms_per_step": round(el3 * 1e3 / steps, 3),
            "acoustic_ms_per_step": round(ac_ms, 3),
            "acoustic_roofline": ac_roof,
            "acoustic_ms_per_step_fast_encoder": round(el_f * 1e3 / steps, 3),
            "host_e2e_ms_per_step": round(el_h * 1e3 / steps, 3),
            "host_e2e_samples_per_s": round(samples / el_h, 1),
            "encoder_precision": "exact (fp32 encoder + variance predictors, GEMMs as 3 f16 MFMAs)",
            "per_gpu_samples_per_s": round(value / ctx.world, 1),
            "x_realtime_per_gpu": round(value / ctx.world / SR, 2), "dtype": "bf16",
            "config": {"workload": "C3 full pipeline (tokens -> FS2-Conformer -> HiFi-GAN), "
                                   f"batch-{B} x {N} tokens x {dur} frames = {T} frames (10.03 s)"},
            "roofline": roofline(prof, el1, steps, "bf16",
                                 (lambda k: pmc_traffic(k, "c3voc_bf16")) if (B, N) == (32, 144) else None,
                                 getattr(ctx, "prof_steps", None))}


def bench_c4(ctx, args, steps, warmup):
    """Config C4: B utterances of mixed length (N_i ~ U{29..144} tokens x 6 frames) owned by rank 0,
    RCCL broadcast -> per-rank length-bucketed synthesis -> RCCL P2P gather to rank 0, all inside
    the timed region (strong scaling: the same 256 utterances whatever N)."""
    from gonova_tts_amd.dist import ShardedSynthesis
    from gonova_tts_amd.model import GonovaTTS
    B = args.c4_batch
    m = GonovaTTS.from_pretrained(ctx.dev.index, vocoder_dtype="bf16", acoustic_dtype="bf16",
                                  max_batch=args.c4_bucket, max_frames=864, max_tokens=144)
    rng = np.random.default_rng(7)
    lens = rng.integers(29, 145, size=B).astype(np.int32)
    tok = np.zeros((B, 144), np.int32)
    for i, L in enumerate(lens):
        tok[i, :L] = rng.integers(1, 78, size=L)

    def synth(t, l):
        d = np.where(np.arange(t.shape[1])[None, :] < l[:, None], 6, 0).astype(np.int32)
        return m.synthesize_tokens(t, l, durations=d, host_lens=False)

    def check(sh):
        out = sh.run(tok if ctx.rank == 0 else None, lens if ctx.rank == 0 else None)
        if ctx.rank == 0:  # every utterance back on the root at its length
            bad = [i for i in range(B) if out[i] is None or out[i].shape[0] != int(lens[i]) * 6 * 256]
            assert not bad, f"C4 gather lost utterances {bad[:8]}"
        return out

    sh = ShardedSynthesis(synth, ctx.dev, bucket=args.c4_bucket)
    run = lambda: sh.run(tok if ctx.rank == 0 else None, lens if ctx.rank == 0 else None)  # noqa: E731
    el1, _ = ctx.timed(run, steps, warmup)
    out1 = check(sh)
    # Two engines per GPU taking the buckets in turn, each on its own stream (dist.py step 4; the
    # service's two-engines-per-GPU shape): one bucket's acoustic pass beside another's vocoder.
    m2 = GonovaTTS.from_pretrained(ctx.dev.index, vocoder_dtype="bf16", acoustic_dtype="bf16",
                                   max_batch=args.c4_bucket, max_frames=864, max_tokens=144)

    def synth2(t, l):
        d = np.where(np.arange(t.shape[1])[None, :] < l[:, None], 6, 0).astype(np.int32)
        return m2.synthesize_tokens(t, l, durations=d, host_lens=False)

    sh2 = ShardedSynthesis([synth, synth2], ctx.dev, bucket=args.c4_bucket)
    run2 = lambda: sh2.run(tok if ctx.rank == 0 else None, lens if ctx.rank == 0 else None)  # noqa: E731
    el2, _ = ctx.timed(run2, steps, warmup)
    out2 = check(sh2)
    if ctx.rank == 0:  # the same bits: an utterance's result does not depend on the engine or bucket
        assert all(np.array_equal(a, b) for a, b in zip(out1, out2)), "C4 two-engine output differs"
    m.engine.close()
    m2.engine.close()
    el = min(el1, el2)
    samples = int(lens.sum()) * 6 * 256 * steps
    value = samples / el
    if ctx.world == 1:
        comm = "single-rank path: no process group, no collective ran (dist.py ShardedSynthesis.single)"
    else:
        comm = f"RCCL broadcast of the tokens + P2P gather of the waveforms to rank 0 over {ctx.world} ranks, inside the timed region"
    return {"value": round(value, 1), "unit": "samples/s", "n_gpus": ctx.world, "scaling": "strong",
            "steps": steps, "warmup": warmup, "ms_per_step": round(el * 1e3 / steps, 3),
            "one_engine_ms_per_step": round(el1 * 1e3 / steps, 3),
            "two_engine_ms_per_step": round(el2 * 1e3 / steps, 3),
            "per_gpu_samples_per_s": round(value / ctx.world, 1),
            "x_realtime_per_gpu": round(value / ctx.world / SR, 2), "dtype": "bf16",
            "config": {"workload": f"C4 batch-{B} mixed-length utterances (N_i ~ U{{29..144}} tokens x 6 frames, "
                                   f"{int(lens.sum()) * 6 * 256 / SR:.0f} s audio), length buckets of "
                                   f"{args.c4_bucket}",
                       "collectives": comm,
                       "bucket_note": "SURVEY.md §8d specifies buckets of 32; 64 measured fastest of 32 / 64 / 128 "
                                      "(BENCH.md) and is the default (--c4-bucket)" if args.c4_bucket != 32 else None,
                       "global_batch": B, "parallelism": f"utterance-sharded dp{ctx.world}"}}


def bench_streaming(ctx, trials=50, B=8, N=144, chunk=32, encoder_precision="exact", predicted=True):
    """Config C5: batch-8 streaming; latency from host tokens to the first audio chunk on host.

    predicted=True (the request path): durations come from the duration predictor (weights with
    the duration linear at w = 0, b = ln 7, so every token gets exactly 6 frames, as C3), then
    the host reads the frame counts (one sync) before the first vocoder chunk.  predicted=False:
    durations given by the caller (stream_tokens(durations=...)): the predictor does not run and
    the frame counts are known on the host without a sync."""
    torch = ctx.torch
    from gonova_tts_amd import model as M
    m = M.GonovaTTS.from_pretrained(ctx.dev.index, vocoder_dtype="bf16", acoustic_dtype="bf16",
                                    encoder_precision=encoder_precision, fixed_duration=6 if predicted else None)
    rng = np.random.default_rng(5)
    tok = rng.integers(1, 78, size=(B, N)).astype(np.int32)
    lens = np.full(B, N, np.int32)
    dur = None if predicted else np.full((B, N), 6, np.int32)
    lat = []
    for i in range(trials + 5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gen = m.stream_tokens(tok, lens, chunk_frames=chunk, durations=dur)
        _, wav, valid = next(gen)
        _ = M._to_host(wav)  # the product's consumer path (GonovaTTS.stream_batch): pinned copy
        t = time.perf_counter() - t0
        gen.close()
        assert int(valid[0]) == chunk * 256
        if i >= 5:
            lat.append(t * 1e3)
    m.engine.close()
    return {"p50_first_audio_ms": round(float(np.percentile(lat, 50)), 3),
            "p90_first_audio_ms": round(float(np.percentile(lat, 90)), 3), "trials": trials,
            "encoder_precision": encoder_precision,
            "durations": "predicted (duration predictor + host read of the frame counts)" if predicted
                         else "given by the caller (predictor skipped, no sync)",
            "config": f"C5 batch-{B} x {N} tokens x 6 frames, chunk {chunk} frames (~{chunk * 256 / SR * 1e3:.0f} ms) "
                      f"+ 16 frames context, bf16"}


def bench_c1(ctx, trials=20):
    """Config C1 (BASELINE.json configs[0]) on the GPU, as the reference serves it: the WebSocket
    service (create_app, the reference's protocol) with the fp32 engine in a TestClient; one
    client sends the 71-token sentence (seeded weights with 6 frames per token: 4.95 s of audio)
    and the time to its first binary frame (= the whole sentence: the reference yields one frame
    per sentence, synthesizer.py:321) and to synthesis_complete is taken over `trials` requests."""
    from fastapi.testclient import TestClient
    from gonova_tts_amd.model import GonovaTTS
    from gonova_tts_amd.service.server import create_app

    def factory():
        return GonovaTTS.from_pretrained(ctx.dev.index, vocoder_dtype="f32", acoustic_dtype="f32", fixed_duration=6)

    first, total, nbytes = [], [], None
    with TestClient(create_app(factory)) as c:
        with c.websocket_connect("/v1/stream/tts") as ws:
            for i in range(trials + 3):
                t0 = time.perf_counter()
                ws.send_text(json.dumps({"type": "synthesize", "text": C1_TEXT, "voice_id": "default"}))
                t_first = None
                while True:
                    msg = ws.receive()
                    if msg.get("bytes") is not None:
                        if t_first is None:
                            t_first = time.perf_counter() - t0
                            nbytes = len(msg["bytes"])
                    elif msg.get("text") is not None:
                        assert json.loads(msg["text"])["type"] == "synthesis_complete"
                        break
                if i >= 3:
                    first.append(t_first * 1e3)
                    total.append((time.perf_counter() - t0) * 1e3)
    samples = nbytes // 4
    assert samples == 71 * 6 * 256, samples
    p50 = float(np.percentile(first, 50))
    return {"p50_first_frame_ms": round(p50, 3), "p90_first_frame_ms": round(float(np.percentile(first, 90)), 3),
            "p50_request_ms": round(float(np.percentile(total, 50)), 3), "trials": trials,
            "samples": samples, "audio_s": round(samples / SR, 3), "rtf": round(p50 * 1e-3 / (samples / SR), 5),
            "dtype": "f32",
            "config": "C1 single 71-token sentence (4.95 s) through the WebSocket service (create_app + TestClient, "
                      "fp32 engine, dynamic batcher), latency from send to the first binary frame"}


def selftest(ctx, args):
    """CPU-only check of the launcher and process group (tests/test_bench_cpu.py): every rank
    contributes its rank to a gloo all-reduce inside the same barrier-bracketed timing."""
    if ctx.rank == args.selftest_fail_rank:
        print(f"bench.py selftest: rank {ctx.rank} exiting on purpose", file=sys.stderr, flush=True)
        os._exit(7)
    t = ctx.torch.tensor([float(ctx.rank)])
    el, _ = ctx.timed(lambda: ctx.dist.all_reduce(t) if ctx.world > 1 else None, 1, 0)
    return {"metric": METRIC, "value": None, "unit": "samples/s", "n_gpus": ctx.world, "steps": 1, "warmup": 0,
            "ms_per_step": round(el * 1e3, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "none", "data": "selftest (no GPU)", "rank_sum": float(t.item()),
            "config": {"workload": "selftest", "parallelism": f"dp{ctx.world}"}}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    ctx = Ctx(args)
    if args.workload == "selftest":
        out = selftest(ctx, args)
    elif args.workload == "c4":
        c = bench_c4(ctx, args, args.steps, args.warmup)
        out = dict({"metric": METRIC}, **c, higher_is_better=True, vs_baseline=None,
                   data="synthetic (token ids U[1,77], N_i ~ U{29..144}, forced 6 frames/token, seeded weights)")
    elif args.workload == "vocoder":
        v = bench_vocoder(ctx, args)
        per_gpu = v["value"] / ctx.world
        out = {
            "metric": METRIC, "value": round(v["value"], 1), "unit": "samples/s", "n_gpus": ctx.world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(v["ms_per_step"], 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (mel ~ N(0,1), seeded fan-in weights; no checkpoint offline)",
            "config": {"workload": f"C2 vocoder-only HiFi-GAN V1, batch-{args.batch} x {args.frames} frames "
                                   f"({args.frames * 256 / SR:.2f} s) per GPU",
                       "global_batch": args.batch * ctx.world, "frames": args.frames,
                       "samples_per_utt": v["samples_per_utt"],
                       "parallelism": f"utterance-sharded dp{ctx.world} (no data-path collective)"},
            "per_gpu_samples_per_s": round(per_gpu, 1),
            "x_realtime_per_gpu": round(per_gpu / SR, 2),
            "rtf": round(SR / per_gpu, 7),
            "algorithmic_tflops_per_gpu": round(v["algorithmic_tflops_per_gpu"], 2),
            "roofline": v["roofline"],
        }
        if not args.no_full:
            out["full_pipeline"] = bench_full(ctx, args, steps=max(3, args.steps // 2), warmup=1)
        if not args.no_c4:
            out["c4"] = bench_c4(ctx, args, steps=max(2, args.steps // 3), warmup=1)
        if not args.no_streaming and ctx.rank == 0:
            out["streaming"] = bench_streaming(ctx)
            for key, kw in (("given_durations", dict(predicted=False)), ("fast_encoder", dict(encoder_precision="fast"))):
                r = bench_streaming(ctx, **kw)
                out["streaming"][key] = {k: r[k] for k in ("p50_first_audio_ms", "p90_first_audio_ms")}
        if not args.no_c1 and ctx.rank == 0 and ctx.world == 1:
            out["c1"] = bench_c1(ctx)
    else:
        f = bench_full(ctx, args, args.steps, args.warmup)
        per_gpu = f["value"] / ctx.world
        out = {"metric": METRIC, "value": f["value"], "unit": "samples/s", "n_gpus": ctx.world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": f["ms_per_step"],
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
               "data": "synthetic (token ids U[1,77], forced 6 frames/token, seeded weights)",
               "config": dict(f["config"], global_batch=args.batch * ctx.world,
                              parallelism=f"utterance-sharded dp{ctx.world}"),
               "per_gpu_samples_per_s": round(per_gpu, 1), "x_realtime_per_gpu": round(per_gpu / SR, 2),
               "rtf": round(SR / per_gpu, 7), "acoustic_ms_per_step": f["acoustic_ms_per_step"],
               "roofline": f["roofline"]}
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline and args.workload != "selftest":
        out["cpu_baseline"] = cpu_baseline(args.cpu_c2_batch, args.cpu_c3_batch)  # rank 0 at N=1 only
    if ctx.rank == 0:
        print(json.dumps(out), flush=True)
    if ctx.world > 1:
        ctx.dist.destroy_process_group()


if __name__ == "__main__":
    main()
