"""Probe: C3 (batch-32 tokens -> FS2-Conformer -> HiFi-GAN, bf16) as one engine on one stream
(the bench line) against two engines on two streams each taking half the batch, so one half's
latency-bound acoustic pass overlaps the other half's MFMA-bound vocoder:
  seq      one engine, B = 32: acoustic then vocoder per step
  conc     two engines, B = 16 each, both halves started together every step
  stagger  two engines, B = 16 each; the second half's stream starts after the first half's
           acoustic pass (one event), so its acoustic pass runs beside the first half's vocoder
  concK    K engines (PROBE_K, default "3,4"), the batch split in K near-equal parts, all started
           together every step, a stream each
  pipe     two engines, whole batches: step i runs batch i's acoustic pass (engine A, stream a)
           beside batch i-1's vocoder (engine B, stream b); both streams joined every step
Prints ms per 32-utterance step (device-resident inputs, 10 timed steps after 3 warmups).

usage (GPU box): python3 tools/c3_overlap_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from gonova_tts_amd.engine import HipEngine
    from gonova_tts_amd.weights import make_acoustic_weights, make_vocoder_weights
    B, N, dur = 32, 144, 6
    T = N * dur
    aw, vw = make_acoustic_weights(seed=0, fixed_duration=dur), make_vocoder_weights(seed=0)
    g = torch.Generator(device="cpu").manual_seed(2000)
    tok = torch.randint(1, 78, (B, N), generator=g, dtype=torch.int32).cuda()
    tl = torch.full((B,), N, dtype=torch.int32, device="cuda")
    wav = torch.empty((B, T * 256), dtype=torch.float32, device="cuda")
    steps = int(os.environ.get("PROBE_STEPS", "10"))

    def timed(fn, warm=3):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / steps

    e1 = HipEngine("cuda:0", vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=B, max_frames=T, max_tokens=N)
    e1.load_weights(vocoder=vw, acoustic=aw)

    def seq():
        mel, ml = e1.acoustic(tok, tl, T)
        e1.vocoder(mel, ml, out=wav)

    t_seq = timed(seq)
    h = B // 2
    e2 = HipEngine("cuda:0", vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=h, max_frames=T, max_tokens=N)
    e2.load_weights(vocoder=vw, acoustic=aw)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    ev = torch.cuda.Event()

    def halves(stagger):
        cur = torch.cuda.current_stream()
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        with torch.cuda.stream(sa):
            mel, ml = e1.acoustic(tok[:h], tl[:h], T, stream=sa)
            if stagger:
                ev.record(sa)
            e1.vocoder(mel, ml, out=wav[:h], stream=sa)
        with torch.cuda.stream(sb):
            if stagger:
                sb.wait_event(ev)
            mel2, ml2 = e2.acoustic(tok[h:], tl[h:], T, stream=sb)
            e2.vocoder(mel2, ml2, out=wav[h:], stream=sb)
        cur.wait_stream(sa)
        cur.wait_stream(sb)

    t_conc = timed(lambda: halves(False))
    t_stag = timed(lambda: halves(True))
    t_seq2 = timed(seq)
    print(f"C3 ms per 32-utterance step: seq {t_seq:.3f} / {t_seq2:.3f}, conc {t_conc:.3f}, stagger {t_stag:.3f}")
    e2.close()
    ea = HipEngine("cuda:0", vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=B, max_frames=T, max_tokens=N)
    ea.load_weights(vocoder=vw, acoustic=aw)
    eb = HipEngine("cuda:0", vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=B, max_frames=T, max_tokens=N)
    eb.load_weights(vocoder=vw, acoustic=aw)
    prev = {}

    def pipe():
        cur = torch.cuda.current_stream()
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        with torch.cuda.stream(sa):
            mel, ml = ea.acoustic(tok, tl, T, stream=sa)
        if prev:
            with torch.cuda.stream(sb):
                eb.vocoder(prev["mel"], prev["ml"], out=wav, stream=sb)
        cur.wait_stream(sa)
        cur.wait_stream(sb)
        prev.update(mel=mel, ml=ml)

    t_p = timed(pipe)
    t_p2 = timed(pipe)
    ref = wav.clone()
    seq()
    torch.cuda.synchronize()
    print(f"C3 ms per 32-utterance step: pipe {t_p:.3f} / {t_p2:.3f} (same waveform as seq: {bool(torch.equal(ref, wav))})")
    ea.close()
    eb.close()
    for k in [int(x) for x in os.environ.get("PROBE_K", "3,4").split(",") if x]:
        cuts = [B * i // k for i in range(k + 1)]
        parts = [slice(cuts[i], cuts[i + 1]) for i in range(k)]
        engs = []
        for sl in parts:
            e = HipEngine("cuda:0", vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=sl.stop - sl.start,
                          max_frames=T, max_tokens=N)
            e.load_weights(vocoder=vw, acoustic=aw)
            engs.append(e)
        sts = [torch.cuda.Stream() for _ in range(k)]

        def conc_k():
            cur = torch.cuda.current_stream()
            for st in sts:
                st.wait_stream(cur)
            for e, st, sl in zip(engs, sts, parts):
                with torch.cuda.stream(st):
                    mel, ml = e.acoustic(tok[sl], tl[sl], T, stream=st)
                    e.vocoder(mel, ml, out=wav[sl], stream=st)
            for st in sts:
                cur.wait_stream(st)

        t_k = timed(conc_k)
        t_k2 = timed(conc_k)
        print(f"C3 ms per 32-utterance step: conc{k} {t_k:.3f} / {t_k2:.3f} ({[sl.stop - sl.start for sl in parts]})")
        for e in engs:
            e.close()
    e1.close()


if __name__ == "__main__":
    main()
