"""GPU tests of the drop-in model surface (from_pretrained / generate / generate_batch),
all through the HIP engine.  The reference's own adapter (core/synthesizer.py) stays the
caller; its contract with the model is pinned by test_generate_contract_matches_reference_call_site."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from gonova_tts_amd.model import GonovaTTS  # noqa: E402
from gonova_tts_amd.text import tokenize  # noqa: E402
from gonova_tts_amd.weights import make_acoustic_weights, make_vocoder_weights  # noqa: E402
from oracle.acoustic import acoustic_forward  # noqa: E402
from oracle.vocoder import vocoder_forward  # noqa: E402


@pytest.fixture(scope="module")
def model32():
    return GonovaTTS.from_pretrained("cuda:0", vocoder_dtype="f32", acoustic_dtype="f32")


def test_generate_contract_matches_reference_call_site(model32):
    audio = model32.generate("Hello world.", audio_prompt_path=None, exaggeration=0.5, cfg_weight=0.5,
                             temperature=0.8, unknown_kwarg=1)
    assert isinstance(audio, torch.Tensor) and audio.dtype == torch.float32 and audio.dim() == 2
    a = audio.squeeze().cpu().numpy()  # reference synthesizer.py:352-353
    assert a.ndim == 1 and a.size % 256 == 0 and np.isfinite(a).all()
    assert model32.sr == 22050


def test_generate_matches_oracle_pipeline(model32):
    text = "The quick brown fox."
    ids = tokenize(text)
    o = acoustic_forward(ids, make_acoustic_weights(0))
    ref = vocoder_forward(o["mel"], make_vocoder_weights(0))
    got = model32.generate(text).squeeze().cpu().numpy()
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, atol=2e-5, rtol=1e-4)


def test_generate_batch_equals_single(model32):
    texts = ["Short one.", "A somewhat longer sentence to synthesize, with a comma.", "Mid length text here."]
    batch = model32.generate_batch(texts)
    for t, b in zip(texts, batch):
        single = model32.generate(t).squeeze().cpu().numpy()
        assert b.shape == single.shape
        np.testing.assert_allclose(b, single, atol=1e-5, rtol=1e-4)


def test_frame_cap_retry_is_exact(model32):
    old = model32.FRAMES_PER_TOKEN_CAP
    try:
        full = model32.generate("Retry path check.").squeeze().cpu().numpy()
        model32.FRAMES_PER_TOKEN_CAP = 1  # force the first pass to truncate
        again = model32.generate("Retry path check.").squeeze().cpu().numpy()
    finally:
        model32.FRAMES_PER_TOKEN_CAP = old
    np.testing.assert_array_equal(full, again)


@pytest.mark.parametrize("dtype", ["f32", "f16"])
def test_streaming_chunks_equal_full_utterance(dtype):
    """Chunked vocoder with 16 frames of context per side reproduces the full pass bit for bit."""
    m = GonovaTTS.from_pretrained("cuda:0", vocoder_dtype=dtype, acoustic_dtype="f32")
    rng = np.random.default_rng(2)
    lens = np.array([60, 33, 47], np.int32)
    tok = np.zeros((3, 60), np.int32)
    for i, L in enumerate(lens):
        tok[i, :L] = rng.integers(1, 78, size=L)
    dur = np.zeros((3, 60), np.int32)
    for i, L in enumerate(lens):
        dur[i, :L] = rng.integers(1, 4, size=L)
    full, full_lens = m.synthesize_tokens(tok, lens, durations=dur)
    full = full.cpu().numpy()
    pieces = [[] for _ in range(3)]
    for c0, wav, valid in m.stream_tokens(tok, lens, chunk_frames=32, durations=dur):
        w = wav.cpu().numpy()
        for b in range(3):
            pieces[b].append(w[b, :valid[b]])
    for b in range(3):
        got = np.concatenate(pieces[b])
        assert got.shape[0] == full_lens[b]
        np.testing.assert_array_equal(got, full[b, :full_lens[b]])


@pytest.mark.parametrize("lens", [[60, 5, 33], [5, 3, 7]])
def test_streaming_predicted_durations_equal_full_utterance(lens):
    """With predicted durations the first chunk is enqueued before the host reads the frame
    counts (used when the longest utterance covers its window, recomputed otherwise: the second
    case, 18-42 frames); the chunks still reproduce the full pass bit for bit."""
    m = GonovaTTS.from_pretrained("cuda:0", vocoder_dtype="f16", acoustic_dtype="bf16", fixed_duration=6)
    rng = np.random.default_rng(3)
    lens = np.array(lens, np.int32)
    tok = np.zeros((3, int(lens.max())), np.int32)
    for i, L in enumerate(lens):
        tok[i, :L] = rng.integers(1, 78, size=L)
    full, full_lens = m.synthesize_tokens(tok, lens)
    full = full.cpu().numpy()
    pieces = [[] for _ in range(3)]
    for c0, wav, valid in m.stream_tokens(tok, lens, chunk_frames=32):
        w = wav.cpu().numpy()
        for b in range(3):
            pieces[b].append(w[b, :valid[b]])
    for b in range(3):
        got = np.concatenate(pieces[b])
        assert got.shape[0] == full_lens[b] == 6 * 256 * lens[b]
        np.testing.assert_array_equal(got, full[b, :full_lens[b]])


def test_generate_at_24khz_is_resampled_native_output(model32):
    """sample_rate=24000 (the rate the reference's clients assume, synthesizer.py:119): the
    22,050 Hz waveform converted on the device == scipy.signal.resample_poly of it."""
    import scipy.signal as ss
    m24 = GonovaTTS(model32.engine, model32.acoustic_cfg, model32.vocoder_cfg, sample_rate=24000)
    assert m24.sr == 24000
    texts = ["Hello world.", "The quick brown fox jumps over the lazy dog."]
    native = model32.generate_batch(texts)
    at24 = m24.generate_batch(texts)
    for a, b in zip(native, at24):
        ref = ss.resample_poly(a.astype(np.float64), 160, 147)
        assert b.shape == ref.shape
        assert np.abs(b - ref).max() <= 2e-6
    one = m24.generate(texts[0]).squeeze().cpu().numpy()
    np.testing.assert_array_equal(one, at24[0])


def test_sharded_synthesis_single_device_matches_direct(model32):
    """dist.ShardedSynthesis on one device (no process group): every bucket is queued before
    the first host sync and the root's audio comes back through per-bucket pinned copies on a
    side stream, overlapped with the next bucket.  Each utterance must equal the same bucket
    synthesized directly (bit for bit) and have the right length; mixed lengths, 3 buckets."""
    from gonova_tts_amd.dist import ShardedSynthesis, plan_buckets
    rng = np.random.default_rng(31)
    lens = rng.integers(5, 40, size=10).astype(np.int32)
    tok = np.zeros((10, 40), np.int32)
    for i, L in enumerate(lens):
        tok[i, :L] = rng.integers(1, 78, size=L)

    def synth(t, l, host_lens=False):
        d = np.where(np.arange(t.shape[1])[None, :] < l[:, None], 3, 0).astype(np.int32)
        return model32.synthesize_tokens(t, l, durations=d, host_lens=host_lens)

    out = ShardedSynthesis(synth, torch.device("cuda:0"), bucket=4).run(tok, lens)
    for bk in plan_buckets(lens, 1, 4)[0]:
        n_b = int(lens[bk].max())
        wav, wl = synth(tok[bk, :n_b], lens[bk], host_lens=True)
        wav = wav.cpu().numpy()
        for j, u in enumerate(bk):
            assert out[u].shape[0] == wl[j] == lens[u] * 3 * 256
            np.testing.assert_array_equal(out[u], wav[j, :wl[j]])


def test_device_bytes_cover_weights_and_workspace():
    """tts_device_bytes (the /health "gpu" figure) counts the engine's own
    device buffers -- at least its weights in their compute dtype plus the vocoder's output-sized
    workspace -- and drops back when the engine closes."""
    from gonova_tts_amd.engine import HipEngine, device_bytes
    torch.cuda.synchronize()
    b0 = device_bytes(0)
    B, T = 8, 200
    eng = HipEngine("cuda:0", vocoder_dtype="f16", acoustic_dtype="bf16", max_batch=B, max_frames=T, max_tokens=40)
    aw, vw = make_acoustic_weights(0), make_vocoder_weights(0)
    eng.load_weights(acoustic=aw, vocoder=vw)
    eng.reserve(B, T, 40)
    b1 = device_bytes(0)
    wbytes = 2 * sum(int(np.asarray(v).size) for v in list(aw.values()) + list(vw.values()))
    work = B * T * 256 * 2  # one fp16 waveform-rate activation buffer of the batch
    print(f"engine device bytes {b1 - b0:,} (weights in 16 bits {wbytes:,}, one activation buffer {work:,})")
    assert b1 - b0 >= wbytes + work
    eng.close()
    assert device_bytes(0) == b0


def test_packed_upload_and_host_read(model32):
    """The request's integer inputs go up as one pinned block (model._upload_i32) and the
    acoustic pass's durations / frame counts / range word come back with one copy
    (model._HostRead over GonovaEngine.acoustic's views): the values equal per-array transfers."""
    from gonova_tts_amd import model as M
    rng = np.random.default_rng(3)
    tok = rng.integers(1, 70, size=(3, 17)).astype(np.int32)
    lens = np.array([17, 9, 1], np.int32)
    dur = rng.integers(0, 5, size=(3, 17)).astype(np.int64)
    empty = np.zeros((2, 0), np.int32)
    t_d, l_d, none_d, d_d, e_d = M._upload_i32((tok, lens, None, dur, empty), "cuda:0")
    assert none_d is None and e_d.shape == (2, 0)
    for a, d in ((tok, t_d), (lens, l_d), (dur, d_d)):
        assert d.dtype == torch.int32 and d.is_contiguous() and tuple(d.shape) == a.shape
        np.testing.assert_array_equal(d.cpu().numpy(), a.astype(np.int32))
    assert t_d.data_ptr() % 64 == 0 and l_d.data_ptr() % 64 == 0 and d_d.data_ptr() % 64 == 0
    eng = model32.engine
    mel, mel_lens, dd, rw = eng.acoustic(t_d, l_d, 12 * 17, return_durations=True, return_range=True)
    one = M._HostRead(dd, mel_lens, rw)
    sep = M._HostRead(dd.clone(), mel_lens.clone(), None if rw is None else rw.clone())
    need1, lens1, tr1 = one.result()
    need2, lens2, tr2 = sep.result()
    assert need1 == need2 and tr1 == tr2
    np.testing.assert_array_equal(lens1, lens2)
    np.testing.assert_array_equal(lens1, mel_lens.cpu().numpy())
    np.testing.assert_array_equal(one.bufs[0].numpy(), dd.cpu().numpy())
