"""GPU parity of the HIP vocoder path (through the C-ABI) against the CPU oracle.

Tolerances: fp32 atol 1e-5 / rtol 1e-4 on the waveform; 16-bit paths
through tests/parity.py (relative RMS and max-abs error, printed and logged, bounded at
about 2x the errors measured on MI355X).
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from gonova_tts_amd.engine import HipEngine, TtsConvDesc, conv1d_op  # noqa: E402
from gonova_tts_amd.weights import make_vocoder_weights  # noqa: E402
from oracle.vocoder import vocoder_forward, conv1d, conv_transpose1d, leaky_relu  # noqa: E402
from parity import check  # noqa: E402

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_v1.npz"))
DEV = "cuda:0"
TDT = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}


def rel_rms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / (np.sqrt(np.mean(b ** 2)) + 1e-30))


@pytest.fixture(scope="module")
def vw():
    return make_vocoder_weights(seed=0)


_ENG = {}


def engine_for(dtype, vw):
    if dtype not in _ENG:
        e = HipEngine(DEV, vocoder_dtype=dtype)
        e.load_weights(vocoder=vw)
        _ENG[dtype] = e
    return _ENG[dtype]


def run_conv(dtype, x, w, b, dil=1, pad=0, x_len=None, in_slope=1.0, act_out=0, r1=None, alpha=1.0,
             out_scale=1.0, y_rows=None):
    """x [B, T, Cin] f32 numpy, w [M, Cin, k] -> y [B, T_out, M] via tts_op_conv1d."""
    B, T, Cin = x.shape
    M, _, k = w.shape
    tout = T + 2 * pad - dil * (k - 1) if y_rows is None else y_rows
    xd = torch.from_numpy(x).to(DEV, TDT[dtype])
    wd = torch.from_numpy(np.ascontiguousarray(w.transpose(0, 2, 1))).to(DEV, TDT[dtype])
    bd = torch.from_numpy(b.astype(np.float32)).to(DEV)
    yd = torch.zeros((B, tout, M), dtype=TDT[dtype], device=DEV)
    lens = torch.tensor(x_len if x_len is not None else [T] * B, dtype=torch.int32, device=DEV)
    ylens = torch.tensor([min(tout, l + 2 * pad - dil * (k - 1)) for l in (x_len or [T] * B)],
                         dtype=torch.int32, device=DEV)
    d = TtsConvDesc()
    d.x, d.sxb, d.sxr, d.x_len, d.x_rows = xd.data_ptr(), T * Cin, Cin, lens.data_ptr(), T
    d.w, d.swb, d.w_ld, d.bias = wd.data_ptr(), 0, k * Cin, bd.data_ptr()
    d.y, d.syb, d.syr = yd.data_ptr(), tout * M, M
    rd = None
    if r1 is not None:
        rd = torch.from_numpy(r1).to(DEV, TDT[dtype])
        d.r1, d.srb, d.srr = rd.data_ptr(), tout * M, M
    d.y_len, d.y_rows = ylens.data_ptr(), tout
    d.M, d.Cin, d.taps, d.dil, d.pad = M, Cin, k, dil, pad
    d.in_slope, d.act_out, d.out_slope, d.alpha, d.out_scale = in_slope, act_out, 0.0, alpha, out_scale
    d.B = B
    conv1d_op(dtype, d)
    torch.cuda.synchronize()
    return yd.float().cpu().numpy()


@pytest.mark.parametrize("Cin,M,k,dil", [(32, 32, 3, 1), (64, 64, 7, 3), (128, 128, 11, 5), (80, 512, 7, 1),
                                         (256, 256, 3, 5), (96, 80, 5, 1), (512, 96, 1, 1)])
def test_conv_op_fp32_matches_oracle(Cin, M, k, dil):
    rng = np.random.default_rng(Cin * 1000 + M + k)
    B, T = 2, 300
    x = rng.standard_normal((B, T, Cin)).astype(np.float32)
    w = (rng.standard_normal((M, Cin, k)) / np.sqrt(Cin * k)).astype(np.float32)
    b = rng.standard_normal(M).astype(np.float32) * 0.1
    pad = dil * (k - 1) // 2
    lens = [T, 177]
    y = run_conv("f32", x, w, b, dil, pad, x_len=lens, in_slope=0.1)
    for i in range(B):
        ref = conv1d(leaky_relu(x[i, :lens[i]], 0.1), w, b, dilation=dil, padding=pad)
        np.testing.assert_allclose(y[i, :lens[i]], ref, atol=2e-5, rtol=1e-4)


def test_conv_op_epilogue_residual_scale():
    rng = np.random.default_rng(7)
    B, T, C = 1, 200, 64
    x = rng.standard_normal((B, T, C)).astype(np.float32)
    r = rng.standard_normal((B, T, C)).astype(np.float32)
    w = (rng.standard_normal((C, C, 3)) / 8).astype(np.float32)
    b = rng.standard_normal(C).astype(np.float32)
    y = run_conv("f32", x, w, b, 1, 1, r1=r, alpha=0.5, act_out=1, out_scale=0.25)
    ref = (np.maximum(0.5 * conv1d(x[0], w, b, padding=1), 0) + r[0]) * 0.25
    np.testing.assert_allclose(y[0], ref, atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize("tag", ["voc_a", "voc_b"])
def test_vocoder_fp32_matches_golden_and_oracle(vw, tag):
    eng = engine_for("f32", vw)
    mel = G[f"{tag}_mel"]
    wav = eng.vocoder(torch.from_numpy(mel)[None].to(DEV)).cpu().numpy()[0]
    np.testing.assert_allclose(wav, G[f"{tag}_wav"], atol=1e-5, rtol=1e-4)
    np.testing.assert_allclose(wav, vocoder_forward(mel, vw), atol=1e-5, rtol=1e-4)


def test_vocoder_fp32_split_layers_range_guard(vw):
    """fp32 vocoders run their 256- and 128-channel resblock convs as split-precision GEMMs
    (round 6; C1).  Their operands must fit f16: with one stage-0 conv scaled by 2e5 the conv after
    it stages values far past 65504, the layers' range word trips, and the engine reruns the forward
    on the fp32 MFMA path by itself -- the waveform is finite (the split form would have staged inf)
    and matches the fp32 oracle of the scaled weights (activations of ~1e5 amplify fp32 rounding
    differences: bar 2e-3 absolute, measured 8.5e-4 on 4 of 6,144 samples, rel-RMS 1e-4)."""
    big = dict(vw)
    big["resblocks.0.convs1.0.weight"] = vw["resblocks.0.convs1.0.weight"] * np.float32(2e5)
    eng = HipEngine(DEV, vocoder_dtype="f32")
    eng.load_weights(vocoder=big)
    mel = G["voc_a_mel"]
    wav = eng.vocoder(torch.from_numpy(mel)[None].to(DEV)).cpu().numpy()[0]
    ref = vocoder_forward(mel, big)
    assert np.isfinite(wav).all()
    err = float(np.abs(wav - ref).max())
    print(f"range-guard fallback: max|err| vs fp32 oracle {err:.2e}, max|ref| {float(np.abs(ref).max()):.3f}")
    np.testing.assert_allclose(wav, ref, atol=2e-3, rtol=1e-2)
    assert rel_rms(wav, ref) < 1e-4
    eng.close()


def test_vocoder_fp32_ragged_batch(vw):
    eng = engine_for("f32", vw)
    rng = np.random.default_rng(5)
    lens = [40, 13, 1, 29]
    T = max(lens)
    mel = rng.standard_normal((len(lens), T, 80)).astype(np.float32)
    wav = eng.vocoder(torch.from_numpy(mel).to(DEV), torch.tensor(lens, dtype=torch.int32)).cpu().numpy()
    for b, L in enumerate(lens):
        ref = vocoder_forward(mel[b, :L], vw)
        np.testing.assert_allclose(wav[b, :L * 256], ref, atol=1e-5, rtol=1e-4)
        assert np.all(wav[b, L * 256:] == 0)


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_vocoder_low_precision_rel_rms(vw, dtype):
    eng = engine_for(dtype, vw)
    rng = np.random.default_rng(11)
    lens = [64, 50]
    mel = rng.standard_normal((2, 64, 80)).astype(np.float32)
    wav = eng.vocoder(torch.from_numpy(mel).to(DEV), torch.tensor(lens, dtype=torch.int32)).cpu().numpy()
    for b, L in enumerate(lens):
        ref = vocoder_forward(mel[b, :L], vw)
        check(f"vocoder {dtype} ragged b={b} ({L} frames)", wav[b, :L * 256], ref, kind="voc_" + dtype)


def test_vocoder_full_size_batch_invariance(vw):
    """C2 shape (B=32, T=862, fp16): every utterance of the batch equals the same
    utterance run alone, bit for bit (size-independent property), and is finite; a window
    of the full-size output itself against the oracle (the vocoder is local: frames
    [w0, w1) from mel frames [w0 - 16, w1 + 16) are exact)."""
    eng = engine_for("f16", vw)
    g = torch.Generator(device="cpu").manual_seed(0)
    mel = torch.randn((32, 862, 80), generator=g).to(DEV)
    wav = eng.vocoder(mel)
    torch.cuda.synchronize()
    assert torch.isfinite(wav).all()
    for b in (0, 17, 31):
        solo = eng.vocoder(mel[b:b + 1].contiguous())
        assert torch.equal(solo[0], wav[b])
    w0, w1 = 100, 300
    ref = vocoder_forward(mel[0, w0 - 16:w1 + 16].cpu().numpy(), vw)[16 * 256:(16 + w1 - w0) * 256]
    check("C2 full-size f16 utt 0 frames 100-300", wav[0, w0 * 256:w1 * 256].cpu().numpy(), ref, kind="voc_f16")


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_fused_mrf_matches_unfused_path(vw, dtype, switch):
    """The fused MRF kernels (ResBlock-pair and resblock-chain launches, the default) against
    the per-conv path (TTS_MRF_FUSED=0) on ragged input."""
    eng = engine_for(dtype, vw)
    rng = np.random.default_rng(21)
    lens = [70, 3, 41, 66]
    mel = torch.from_numpy(rng.standard_normal((4, 70, 80)).astype(np.float32)).to(DEV)
    ln = torch.tensor(lens, dtype=torch.int32)
    switch("TTS_MRF_FUSED", 1)
    fused = eng.vocoder(mel, ln).cpu().numpy()
    switch("TTS_MRF_FUSED", 0)
    unfused = eng.vocoder(mel, ln).cpu().numpy()
    for b, L in enumerate(lens):
        e = rel_rms(fused[b, :L * 256], unfused[b, :L * 256])
        assert e <= (2e-3 if dtype == "f16" else 1.5e-2), (b, e)
        assert np.all(fused[b, L * 256:] == 0)


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_resblock_chain_bit_identical_to_pairs(vw, dtype, switch):
    """The resblock chain kernel (three pairs in one launch: k=3 at C=32/64, k=7 at C=32)
    reproduces the three pair launches bit for bit, ragged utterances and tile edges included
    (first / last blocks of an utterance, one block shorter than the halo)."""
    eng = engine_for(dtype, vw)
    rng = np.random.default_rng(22)
    lens = [70, 1, 33, 64, 5]
    mel = torch.from_numpy(rng.standard_normal((5, 70, 80)).astype(np.float32)).to(DEV)
    ln = torch.tensor(lens, dtype=torch.int32)
    switch("TTS_MRF_FUSED", 1)
    switch("TTS_MRF_CHAIN", 1)
    chain = eng.vocoder(mel, ln).cpu().numpy()
    switch("TTS_MRF_CHAIN", 0)
    pairs = eng.vocoder(mel, ln).cpu().numpy()
    for b, L in enumerate(lens):
        assert np.array_equal(chain[b], pairs[b]), (b, float(np.abs(chain[b] - pairs[b]).max()))
        assert np.all(chain[b, L * 256:] == 0)


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_fused_conv_post_bit_identical(vw, dtype, switch):
    """conv_post inside the last pair launch (its halo rows computed in the block, the final
    MRF sum never written) reproduces the separate conv_post launch bit for bit: ragged and
    empty utterances, a batch length that is not a whole number of 512-row tiles, utterances
    shorter than one tile, and the zero tail past every utterance."""
    eng = engine_for(dtype, vw)
    rng = np.random.default_rng(23)
    lens = [71, 1, 2, 0, 33, 64]
    mel = torch.from_numpy(rng.standard_normal((6, 71, 80)).astype(np.float32)).to(DEV)
    ln = torch.tensor(lens, dtype=torch.int32)
    switch("TTS_POST_FUSE", 1)
    fused = eng.vocoder(mel, ln).cpu().numpy()
    switch("TTS_POST_FUSE", 0)
    sep = eng.vocoder(mel, ln).cpu().numpy()
    for b, L in enumerate(lens):
        assert np.array_equal(fused[b], sep[b]), (b, float(np.abs(fused[b] - sep[b]).max()))
        assert np.all(fused[b, L * 256:] == 0)


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_short_pair_tiles_bit_identical(vw, dtype, switch):
    """Short pair tiles (picked for grids that leave most CUs idle, e.g. the streamed vocoder's
    stage 0) reproduce the full-height tiles bit for bit at every C (forced), ragged and empty
    utterances and tile edges included; the automatic choice agrees too."""
    eng = engine_for(dtype, vw)
    rng = np.random.default_rng(24)
    lens = [71, 1, 0, 33, 64]
    mel = torch.from_numpy(rng.standard_normal((5, 71, 80)).astype(np.float32)).to(DEV)
    ln = torch.tensor(lens, dtype=torch.int32)
    switch("TTS_MRF_CHAIN", 0)     # every resblock as pair launches
    switch("TTS_PAIR_SPLIT", 0)    # (the channel-split form has its own test below)
    switch("TTS_PAIR_DIV", 0)
    short = eng.vocoder(mel, ln).cpu().numpy()
    switch("TTS_PAIR_DIV", 1)
    full = eng.vocoder(mel, ln).cpu().numpy()
    switch("TTS_MRF_CHAIN", None)
    default_full = eng.vocoder(mel, ln).cpu().numpy()
    switch("TTS_PAIR_DIV", None)
    auto = eng.vocoder(mel, ln).cpu().numpy()
    for b, L in enumerate(lens):
        assert np.array_equal(short[b], full[b]), (b, float(np.abs(short[b] - full[b]).max()))
        assert np.array_equal(auto[b], default_full[b]), b
        assert np.all(short[b, L * 256:] == 0)


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_channel_split_pairs_bit_identical(vw, dtype, switch):
    """The channel-split pair form (two launches per pair over (row tile, 64-channel slice)
    blocks, t rows through the T1 scratch; picked for small C >= 128 grids such as the streamed
    vocoder's first chunk) reproduces mrf_pair_kernel bit for bit: forced on and off, ragged and
    empty utterances, tile edges, the stage-final pairs with the stored LeakyReLU included; the
    automatic choice agrees, and the zero tail past each utterance stays zero."""
    eng = engine_for(dtype, vw)
    rng = np.random.default_rng(25)
    lens = [71, 1, 0, 33, 64, 8]
    mel = torch.from_numpy(rng.standard_normal((6, 71, 80)).astype(np.float32)).to(DEV)
    ln = torch.tensor(lens, dtype=torch.int32)
    switch("TTS_MRF_CHAIN", 0)     # every resblock as pair launches
    outs = {}
    for sp, div in ((0, 1), (1, 1), (None, 1), (0, None), (1, None), (None, None)):
        switch("TTS_PAIR_SPLIT", sp)
        switch("TTS_PAIR_DIV", div)
        outs[(sp, div)] = eng.vocoder(mel, ln).cpu().numpy()
    switch("TTS_MRF_CHAIN", None)
    switch("TTS_PAIR_SPLIT", 1)
    chain_split = eng.vocoder(mel, ln).cpu().numpy()
    switch("TTS_PAIR_SPLIT", 0)
    chain_full = eng.vocoder(mel, ln).cpu().numpy()
    ref = outs[(0, 1)]
    for k, o in outs.items():
        for b, L in enumerate(lens):
            assert np.array_equal(o[b], ref[b]), (k, b, float(np.abs(o[b] - ref[b]).max()))
            assert np.all(o[b, L * 256:] == 0), (k, b)
    assert np.array_equal(chain_split, chain_full)


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_streaming_upsampler_matches_conv_path(vw, dtype, switch):
    """The streaming transposed-conv kernel of stages 2-3 (weights in LDS, B fragments straight
    from HBM, zero rows outside each utterance through the buffer descriptor) against the
    conv_xres polyphase path and the oracle: ragged and empty utterances, lengths that end
    mid-item; the zero tail past each utterance stays zero."""
    eng = engine_for(dtype, vw)
    rng = np.random.default_rng(24)
    lens = [45, 1, 0, 17, 32]
    mel = torch.from_numpy(rng.standard_normal((5, 45, 80)).astype(np.float32)).to(DEV)
    ln = torch.tensor(lens, dtype=torch.int32)
    switch("TTS_UP_STREAM", 1)
    st = eng.vocoder(mel, ln).cpu().numpy()
    switch("TTS_UP_STREAM", 0)
    cv = eng.vocoder(mel, ln).cpu().numpy()
    tol = 2e-3 if dtype == "f16" else 1.5e-2
    for b, L in enumerate(lens):
        if L:
            assert rel_rms(st[b, :L * 256], cv[b, :L * 256]) <= tol, b
        assert np.all(st[b, L * 256:] == 0)
    ref = vocoder_forward(mel[3, :17].cpu().numpy(), vw)
    check(f"streaming upsampler {dtype} 17 frames", st[3, :17 * 256], ref, kind="voc_" + dtype)


@pytest.mark.parametrize("dtype", ["f32", "f16", "bf16"])
def test_zero_length_utterance_in_batch(vw, dtype):
    """An empty utterance (0 frames) inside a ragged batch yields all-zero audio and leaves the
    other utterances exactly as when run alone (every launch masks per utterance)."""
    eng = engine_for(dtype, vw)
    rng = np.random.default_rng(31)
    lens = [0, 19, 0, 7]
    mel = torch.from_numpy(rng.standard_normal((4, 19, 80)).astype(np.float32)).to(DEV)
    wav = eng.vocoder(mel, torch.tensor(lens, dtype=torch.int32)).cpu()
    assert torch.all(wav[0] == 0) and torch.all(wav[2] == 0)
    for b in (1, 3):
        solo = eng.vocoder(mel[b:b + 1, :lens[b]].contiguous()).cpu()
        assert torch.equal(wav[b, :lens[b] * 256], solo[0])
        assert torch.all(wav[b, lens[b] * 256:] == 0)


def test_long_utterance_matches_oracle_slice(vw):
    """A 2,600-frame (30 s) utterance: the fp16 default path against the oracle on a window
    whose receptive field lies inside the utterance (a slice of the full oracle run would
    take minutes on the CPU; the vocoder is local, so the window is exact up to its edges)."""
    eng = engine_for("f16", vw)
    rng = np.random.default_rng(32)
    T = 2600
    mel = rng.standard_normal((1, T, 80)).astype(np.float32)
    wav = eng.vocoder(torch.from_numpy(mel).to(DEV)).cpu().numpy()[0]
    assert wav.shape == (T * 256,) and np.isfinite(wav).all()
    w0, w1, ctx = 1800, 1840, 16  # compare frames [w0, w1) computed from frames [w0-ctx, w1+ctx)
    ref = vocoder_forward(mel[0, w0 - ctx:w1 + ctx], vw)[ctx * 256:(ctx + w1 - w0) * 256]
    check("long 2600-frame f16 frames 1800-1840", wav[w0 * 256:w1 * 256], ref, kind="voc_f16")


def test_bad_arguments_raise_with_the_engine_message(vw):
    """Errors cross the C-ABI as codes + tts_last_error text and surface as RuntimeError
    (the reference re-raises model exceptions, synthesizer.py:323-325)."""
    import ctypes
    eng = engine_for("f16", vw)
    rc = eng.lib.tts_vocoder_forward(eng.handle, None, None, 0, 10, None, None)
    assert rc != 0
    assert eng.lib.tts_last_error()
    with pytest.raises(RuntimeError):
        eng.resample(torch.zeros((1, 8), device=DEV), torch.tensor([8], dtype=torch.int32), 0, 1)
    del ctypes


def test_two_streams_share_one_engine(vw):
    """Calls on two streams of one engine share its workspace; the engine orders a call on a
    new stream after everything the previous call's stream enqueued (event edge), so results
    equal single-stream runs bit for bit (advisor finding: cross-stream scratch race)."""
    eng = engine_for("f16", vw)
    rng = np.random.default_rng(41)
    melA = torch.from_numpy(rng.standard_normal((4, 120, 80)).astype(np.float32)).to(DEV)
    melB = torch.from_numpy(rng.standard_normal((3, 90, 80)).astype(np.float32)).to(DEV)
    refA, refB = eng.vocoder(melA).clone(), eng.vocoder(melB).clone()
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for _ in range(3):
        with torch.cuda.stream(s1):
            a = eng.vocoder(melA, stream=s1)
        with torch.cuda.stream(s2):
            b = eng.vocoder(melB, stream=s2)
        outs.append((a, b))
    torch.cuda.synchronize()
    for a, b in outs:
        assert torch.equal(a, refA) and torch.equal(b, refB)


def test_caller_stream_destroyed_between_calls(vw):
    """A C caller may destroy its per-request stream as soon as a call returns (advisor finding:
    the engine used to record its ordering event on the PREVIOUS call's stream at the start of
    the next call).  Stream A runs a forward and is destroyed; the next call, on another
    stream, must succeed and match, and so must a third on a fresh stream."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]

    class RawStream:  # what engine._stream_ptr reads from a torch stream
        def __init__(self):
            self.ptr = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(self.ptr)) == 0
            self.cuda_stream = self.ptr.value

    eng = engine_for("f16", vw)
    rng = np.random.default_rng(43)
    mel = torch.from_numpy(rng.standard_normal((2, 64, 80)).astype(np.float32)).to(DEV)
    ref = eng.vocoder(mel).clone()
    torch.cuda.synchronize()
    a = RawStream()
    outA = eng.vocoder(mel, stream=a)
    assert hip.hipStreamSynchronize(a.ptr) == 0
    assert hip.hipStreamDestroy(a.ptr) == 0
    outB = eng.vocoder(mel)  # torch's current stream: a different stream than A
    torch.cuda.synchronize()
    c = RawStream()
    outC = eng.vocoder(mel, stream=c)
    assert hip.hipStreamSynchronize(c.ptr) == 0
    assert hip.hipStreamDestroy(c.ptr) == 0
    assert torch.equal(outA, ref) and torch.equal(outB, ref) and torch.equal(outC, ref)
