"""GPU parity of the benchmarked configurations themselves (BASELINE.json configs[2..4]),
through the C-ABI, against the CPU oracle (oracle/acoustic.py + oracle/vocoder.py).

* C3: tokens -> bf16 acoustic -> bf16 vocoder, 144 tokens x 6 frames (duration linear w = 0,
  b = ln 7), composed exactly as bench.py times it.  Oracle parity on a batch
  of 4 (whole mel + a 2 s waveform window), and the full B = 32 x 864 batch through
  size-independent properties (every mel length 864, finite, each utterance bit-identical to
  the same utterance run alone).
* C5: the streamed vocoder at bf16, batch 8, 32-frame chunks with 16 frames of context:
  chunks bit-identical to the full pass, the full pass against the oracle on a window.
* C2: a window of the B = 32 x 862 fp16 run itself against the oracle.

The vocoder is local (receptive field < 13 frames per side), so the oracle waveform of frames
[w0, w1) computed from mel frames [w0 - 16, w1 + 16) equals its full-utterance waveform there:
a window comparison is exact up to rounding while the full oracle run would take minutes.
Tolerances: tests/parity.py (about 2x the MI355X-measured errors)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from parity import check  # noqa: E402

from gonova_tts_amd.engine import HipEngine  # noqa: E402
from gonova_tts_amd.model import GonovaTTS  # noqa: E402
from gonova_tts_amd.weights import make_acoustic_weights, make_vocoder_weights  # noqa: E402
from oracle.acoustic import acoustic_forward  # noqa: E402
from oracle.vocoder import vocoder_forward  # noqa: E402

DEV = "cuda:0"
CTX = 16
HOP = 256


def oracle_window(mel, w0, w1, vw):
    """Oracle waveform of frames [w0, w1) of the utterance with mel [T, 80] (exact: local)."""
    a, b = max(0, w0 - CTX), min(mel.shape[0], w1 + CTX)
    return vocoder_forward(mel[a:b], vw)[(w0 - a) * HOP:(w1 - a) * HOP]


# ----------------------------------------------------------------------------- C3
@pytest.fixture(scope="module")
def c3():
    aw = make_acoustic_weights(seed=0, fixed_duration=6)
    vw = make_vocoder_weights(seed=0)
    eng = HipEngine(DEV, vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=32, max_frames=864, max_tokens=144)
    eng.load_weights(vocoder=vw, acoustic=aw)
    rng = np.random.default_rng(2000)
    tok = rng.integers(1, 78, size=(32, 144)).astype(np.int32)
    return eng, aw, vw, tok


def c3_run(eng, tok):
    B = tok.shape[0]
    t = torch.from_numpy(tok).to(DEV)
    tl = torch.full((B,), 144, dtype=torch.int32, device=DEV)
    mel, mel_lens = eng.acoustic(t, tl, 864)
    wav = eng.vocoder(mel, mel_lens)
    torch.cuda.synchronize()
    return mel.cpu().numpy(), mel_lens.cpu().numpy(), wav.cpu().numpy()


def test_c3_pipeline_matches_oracle(c3):
    eng, aw, vw, tok = c3
    mel, mel_lens, wav = c3_run(eng, tok[:4])
    assert np.all(mel_lens == 864)
    for b in range(4):
        ref = acoustic_forward(tok[b], aw)
        assert np.all(ref["durations"] == 6)
        check(f"C3.mel[b={b}] bf16", mel[b], ref["mel"], kind="ac_bf16")
        w0, w1 = 300, 472  # 2 s
        got = wav[b, w0 * HOP:w1 * HOP]
        check(f"C3.wav[b={b}] bf16 frames {w0}-{w1}", got, oracle_window(ref["mel"], w0, w1, vw), kind="e2e_bf16")
        # the vocoder alone on the engine's own mel: isolates the bf16 vocoder error
        check(f"C3.vocoder-only[b={b}] bf16", got, oracle_window(mel[b], w0, w1, vw), kind="voc_bf16")


def test_c3_full_size_batch_properties(c3):
    eng, aw, vw, tok = c3
    mel, mel_lens, wav = c3_run(eng, tok)
    assert mel.shape == (32, 864, 80) and wav.shape == (32, 864 * HOP)
    assert np.all(mel_lens == 864)
    assert np.isfinite(mel).all() and np.isfinite(wav).all()
    for b in (0, 13, 31):
        m1, l1, w1 = c3_run(eng, tok[b:b + 1])
        assert np.array_equal(m1[0], mel[b]), b
        assert np.array_equal(w1[0], wav[b]), b


# ----------------------------------------------------------------------------- C5
def test_c5_streaming_bf16_batch8_bit_identical_and_matches_oracle():
    m = GonovaTTS.from_pretrained(DEV, vocoder_dtype="bf16", acoustic_dtype="bf16")
    rng = np.random.default_rng(5)
    B, N = 8, 144
    tok = rng.integers(1, 78, size=(B, N)).astype(np.int32)
    lens = np.full(B, N, np.int32)
    lens[3] = 101  # one ragged utterance: its stream ends mid-window
    tok[3, 101:] = 0
    dur = np.where(np.arange(N)[None, :] < lens[:, None], 6, 0).astype(np.int32)
    full, full_lens = m.synthesize_tokens(tok, lens, durations=dur)
    full = full.cpu().numpy()
    pieces = [[] for _ in range(B)]
    n_chunks = 0
    for c0, wav, valid in m.stream_tokens(tok, lens, chunk_frames=32, context=16, durations=dur):
        w = wav.cpu().numpy()
        n_chunks += 1
        for b in range(B):
            pieces[b].append(w[b, :valid[b]])
    assert n_chunks == 27  # 864 frames / 32
    for b in range(B):
        got = np.concatenate(pieces[b])
        assert got.shape[0] == full_lens[b] == lens[b] * 6 * HOP
        assert np.array_equal(got, full[b, :full_lens[b]]), b
    aw, vw = make_acoustic_weights(0), make_vocoder_weights(0)
    for b in (0, 3):
        ref = acoustic_forward(tok[b, :lens[b]], aw, durations=dur[b, :lens[b]])
        for w0, w1 in ((0, 32), (200, 372)):  # the first chunk, and 2 s mid-utterance
            check(f"C5.wav[b={b}] bf16 frames {w0}-{w1}", full[b, w0 * HOP:w1 * HOP],
                  oracle_window(ref["mel"], w0, w1, vw), kind="e2e_bf16")
    m.engine.close()


# ----------------------------------------------------------------------------- C2
def test_c2_full_size_window_matches_oracle():
    """The C2 batch itself (B = 32 x 862, fp16, full-height pair tiles): windows of its
    utterances against the oracle (start, middle and end of the utterance)."""
    vw = make_vocoder_weights(seed=0)
    eng = HipEngine(DEV, vocoder_dtype="f16")
    eng.load_weights(vocoder=vw)
    g = torch.Generator(device="cpu").manual_seed(1000)
    mel = torch.randn((32, 862, 80), generator=g)
    wav = eng.vocoder(mel.to(DEV)).cpu().numpy()
    mel = mel.numpy()
    for b, (w0, w1) in ((0, (0, 40)), (17, (400, 440)), (31, (822, 862))):
        check(f"C2.wav[b={b}] f16 frames {w0}-{w1}", wav[b, w0 * HOP:w1 * HOP],
              oracle_window(mel[b], w0, w1, vw), kind="voc_f16")
    eng.close()


# ----------------------------------------------------------------------------- C4
def test_c4_sharded_batch256_matches_solo_and_oracle():
    """C4 itself (BASELINE.json configs[3]): 256 utterances of N_i ~ U{29..144} tokens x 6
    frames, length buckets of 64, bf16, through dist.ShardedSynthesis exactly as bench.py runs
    it -- once inside an RCCL process group (backend "nccl" = RCCL, one rank on this 1-GPU box:
    the token broadcast runs as an RCCL collective and the gather's CPU metadata group is created;
    the P2P gather has no peer here, tests/test_dist_cpu.py covers it with gloo ranks) and once
    with no group.
    Checks: every utterance returns at 6 * 256 * N_i samples, both runs agree bit for bit,
    8 utterances (shortest, longest and 6 between) equal the same utterance synthesized alone
    bit for bit, and 2 match the oracle on 2 s windows."""
    import datetime
    import socket

    import torch.distributed as dist

    from gonova_tts_amd.dist import ShardedSynthesis

    B, bucket = 256, 64
    m = GonovaTTS.from_pretrained(DEV, vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=bucket,
                                  max_frames=864, max_tokens=144)
    rng = np.random.default_rng(7)  # bench.py's C4 draw
    lens = rng.integers(29, 145, size=B).astype(np.int32)
    tok = np.zeros((B, 144), np.int32)
    for i, L in enumerate(lens):
        tok[i, :L] = rng.integers(1, 78, size=L)

    def durs(t, l):
        return np.where(np.arange(t.shape[1])[None, :] < l[:, None], 6, 0).astype(np.int32)

    def synth(t, l):
        return m.synthesize_tokens(t, l, durations=durs(t, l), host_lens=False)

    plain = ShardedSynthesis(synth, torch.device(DEV), bucket=bucket).run(tok, lens)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            timeout=datetime.timedelta(seconds=60), device_id=torch.device(DEV))
    try:
        sh = ShardedSynthesis(synth, torch.device(DEV), bucket=bucket)
        assert not sh.single and sh.world == 1
        out = sh.run(tok, lens)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    for i in range(B):
        assert out[i] is not None and out[i].shape == (int(lens[i]) * 6 * HOP,), i
        assert np.isfinite(out[i]).all(), i
        assert np.array_equal(out[i], plain[i]), i
    order = np.argsort(lens, kind="stable")
    picks = [int(order[j]) for j in np.linspace(0, B - 1, 8).round().astype(int)]
    for u in picks:
        L = int(lens[u])
        solo, solo_lens = m.synthesize_tokens(tok[u:u + 1, :L], lens[u:u + 1], durations=durs(tok[u:u + 1, :L], lens[u:u + 1]))
        solo = solo.cpu().numpy()[0, :int(solo_lens[0])]
        assert np.array_equal(out[u], solo), (u, L, float(np.abs(out[u] - solo).max()))
    aw, vw = make_acoustic_weights(0), make_vocoder_weights(0)
    for u in (picks[0], picks[-1]):  # the shortest and the longest utterance
        L = int(lens[u])
        ref = acoustic_forward(tok[u, :L], aw, durations=np.full(L, 6, np.int32))
        w1 = L * 6
        w0 = w1 - 172  # the last 2 s, through the utterance's end
        check(f"C4.wav[u={u}, N={L}] bf16 frames {w0}-{w1}", out[u][w0 * HOP:w1 * HOP],
              oracle_window(ref["mel"], w0, w1, vw), kind="e2e_bf16")
    m.engine.close()


def test_c3_pipelined_form_matches_one_stream():
    """bench.py's pipelined C3 form -- each step runs batch k's acoustic pass (engine A, stream a)
    beside batch k-1's vocoder (engine B, stream b) -- writes the same waveform bits as the
    one-stream step, for batches that differ from step to step."""
    B, N, dur = 4, 32, 6
    T = N * dur
    aw, vw = make_acoustic_weights(seed=0, fixed_duration=dur), make_vocoder_weights(seed=0)
    engs = []
    for _ in range(2):
        e = HipEngine(DEV, vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=B, max_frames=T, max_tokens=N)
        e.load_weights(vocoder=vw, acoustic=aw)
        engs.append(e)
    ea, eb = engs
    g = torch.Generator(device="cpu").manual_seed(11)
    toks = [torch.randint(1, 78, (B, N), generator=g, dtype=torch.int32).to(DEV) for _ in range(3)]
    tl = torch.full((B,), N, dtype=torch.int32, device=DEV)
    ref = []
    for tok in toks:
        mel, ml = ea.acoustic(tok, tl, T)
        ref.append(ea.vocoder(mel, ml).clone())
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    outs, prev = [], None
    for tok in toks + [None]:
        cur = torch.cuda.current_stream()
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        nxt = None
        if tok is not None:
            with torch.cuda.stream(sa):
                nxt = ea.acoustic(tok, tl, T, stream=sa)
        if prev is not None:
            with torch.cuda.stream(sb):
                outs.append(eb.vocoder(prev[0], prev[1], stream=sb))
        cur.wait_stream(sa)
        cur.wait_stream(sb)
        prev = nxt
    torch.cuda.synchronize()
    for e in engs:
        e.close()
    assert len(outs) == len(ref)
    for o, r in zip(outs, ref):
        assert torch.equal(o, r)
