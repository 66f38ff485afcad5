"""GPU parity of the HIP acoustic model (FastSpeech2-Conformer, through the C-ABI)
against the CPU oracle and the transformers golden vectors.

Tolerances: fp32 mel atol 1e-5 / rtol 1e-4 (FP32_ATOL / FP32_RTOL below: SURVEY.md §8c's fp32
bar; measured max error 6.0e-6, profiles/r04zc_fp32_mel_error.txt); durations exact (except a
logit within 1e-3 of a rounding boundary); 16-bit mel through tests/parity.py (rel-RMS and
max-abs, ~2x the measured error) with durations forced.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from gonova_tts_amd.engine import HipEngine  # noqa: E402
from gonova_tts_amd.weights import make_acoustic_weights, make_vocoder_weights  # noqa: E402
from oracle.acoustic import acoustic_forward  # noqa: E402
from oracle.vocoder import vocoder_forward  # noqa: E402
from parity import check  # noqa: E402

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_v1.npz"))
DEV = "cuda:0"


def rel_rms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / (np.sqrt(np.mean(b ** 2)) + 1e-30))


# fp32 mel against the transformers goldens / the oracle: SURVEY.md §8c's fp32 bars.  Measured
# (tools/fp32_err_probe.py, round 4): max abs error 4.9e-6 .. 6.0e-6, rel-RMS 1.3e-6 .. 1.6e-6.
FP32_ATOL, FP32_RTOL = 1e-5, 1e-4


@pytest.fixture(scope="module")
def aw():
    return make_acoustic_weights(seed=0)


_ENG = {}


def engine(dtype, aw, vocoder=False):
    key = (dtype, vocoder)
    if key not in _ENG:
        e = HipEngine(DEV, vocoder_dtype="f32", acoustic_dtype=dtype)
        e.load_weights(acoustic=aw, vocoder=make_vocoder_weights(seed=0) if vocoder else None)
        _ENG[key] = e
    return _ENG[key]


def run(eng, ids_list, t_cap, durations=None):
    B = len(ids_list)
    N = max(len(x) for x in ids_list)
    tok = np.zeros((B, N), np.int32)
    for b, x in enumerate(ids_list):
        tok[b, :len(x)] = x
    lens = torch.tensor([len(x) for x in ids_list], dtype=torch.int32)
    dd = None
    if durations is not None:
        d = np.zeros((B, N), np.int32)
        for b, x in enumerate(durations):
            d[b, :len(x)] = x
        dd = torch.from_numpy(d).to(DEV)
    mel, mel_lens, dur = eng.acoustic(torch.from_numpy(tok).to(DEV), lens, t_cap, durations=dd,
                                      return_durations=True)
    torch.cuda.synchronize()
    return mel.cpu().numpy(), mel_lens.cpu().numpy(), dur.cpu().numpy()


@pytest.mark.parametrize("tag", ["ac_a", "ac_b"])
def test_acoustic_fp32_matches_golden(aw, tag):
    eng = engine("f32", aw)
    ids = G[f"{tag}_ids"]
    mel, mel_lens, dur = run(eng, [ids], t_cap=128)
    np.testing.assert_array_equal(dur[0, :len(ids)], G[f"{tag}_dur"])
    L = int(mel_lens[0])
    assert L == G[f"{tag}_mel"].shape[0]
    np.testing.assert_allclose(mel[0, :L], G[f"{tag}_mel"], atol=FP32_ATOL, rtol=FP32_RTOL)
    assert np.all(mel[0, L:] == 0)


def test_acoustic_fp32_ragged_batch_matches_oracle(aw):
    eng = engine("f32", aw)
    rng = np.random.default_rng(3)
    ids_list = [rng.integers(1, 78, size=n) for n in (20, 7, 33, 1)]
    mel, mel_lens, dur = run(eng, ids_list, t_cap=200)
    skipped = []
    for b, ids in enumerate(ids_list):
        ref = acoustic_forward(ids, aw)
        # durations: exact unless the oracle's exp(x)-1 is within 1e-3 of a .5 rounding boundary
        frac = np.abs((np.exp(ref["log_durations"]) - 1) % 1 - 0.5)
        ok = frac > 1e-3
        np.testing.assert_array_equal(dur[b, :len(ids)][ok], ref["durations"][ok])
        if not np.array_equal(dur[b, :len(ids)], ref["durations"]):
            skipped.append(b)  # a boundary token rounded the other way: the frame grids differ
            continue
        L = int(mel_lens[b])
        assert L == min(ref["mel"].shape[0], 200)
        np.testing.assert_allclose(mel[b, :L], ref["mel"][:L], atol=FP32_ATOL, rtol=FP32_RTOL)
    # the mel comparison may skip at most one utterance (a 1e-3 boundary case), never the batch
    assert len(skipped) <= 1, skipped


def test_acoustic_fp32_split_k_batch_invariant(aw):
    """The fp32 model's GEMMs split K on a workspace with a slice count from the layer shape only
    (conv_gemm.hip f32_kslices): an utterance's durations and mel are bit-identical whether it runs
    alone (batch-1 grids: the split-K form) or inside a ragged batch of four."""
    eng = engine("f32", aw)
    rng = np.random.default_rng(17)
    ids_list = [rng.integers(1, 78, size=n) for n in (41, 9, 71, 26)]
    mel, mel_lens, dur = run(eng, ids_list, t_cap=12 * 71)
    for b, ids in enumerate(ids_list):
        m1, l1, d1 = run(eng, [ids], t_cap=12 * 71)
        assert int(l1[0]) == int(mel_lens[b])
        assert np.array_equal(d1[0, :len(ids)], dur[b, :len(ids)])
        L = int(l1[0])
        assert np.array_equal(m1[0, :L], mel[b, :L]), b


def test_acoustic_duration_override_and_cap(aw):
    eng = engine("f32", aw)
    rng = np.random.default_rng(9)
    ids = rng.integers(1, 78, size=15)
    d = rng.integers(0, 5, size=15)
    mel, mel_lens, dur = run(eng, [ids], t_cap=256, durations=[d])
    ref = acoustic_forward(ids, aw, durations=d)
    np.testing.assert_array_equal(dur[0, :15], d)
    assert int(mel_lens[0]) == int(d.sum())
    np.testing.assert_allclose(mel[0, :int(d.sum())], ref["mel"], atol=FP32_ATOL, rtol=FP32_RTOL)
    # cap: frames beyond Tcap are dropped, the kept prefix is unchanged
    cap = int(d.sum()) - 5
    mel2, mel_lens2, _ = run(eng, [ids], t_cap=cap, durations=[d])
    assert int(mel_lens2[0]) == cap
    ref2 = acoustic_forward(ids, aw, durations=d)  # decoder sees only cap frames on GPU
    assert np.all(np.isfinite(mel2[0, :cap]))
    # all-zero durations -> one frame per token (HF:108-109, per utterance)
    mel3, mel_lens3, dur3 = run(eng, [ids], t_cap=64, durations=[np.zeros(15, np.int64)])
    assert int(mel_lens3[0]) == 15 and np.all(dur3[0, :15] == 1)
    del ref2


def test_acoustic_bf16_forced_durations(aw):
    eng = engine("bf16", aw)
    rng = np.random.default_rng(4)
    ids_list = [rng.integers(1, 78, size=n) for n in (40, 25)]
    durs = [np.full(len(x), 6) for x in ids_list]
    mel, mel_lens, _ = run(eng, ids_list, t_cap=240, durations=durs)
    for b, ids in enumerate(ids_list):
        ref = acoustic_forward(ids, aw, durations=durs[b])
        L = int(mel_lens[b])
        assert L == len(ids) * 6
        check(f"acoustic bf16 forced-dur b={b}", mel[b, :L], ref["mel"], kind="ac_bf16")


def test_end_to_end_fp32_matches_golden(aw):
    eng = engine("f32", aw, vocoder=True)
    ids = G["ac_a_ids"]
    mel, mel_lens, _ = run(eng, [ids], t_cap=64)
    L = int(mel_lens[0])
    wav = eng.vocoder(torch.from_numpy(mel[:, :L].copy()).to(DEV)).cpu().numpy()[0]
    np.testing.assert_allclose(wav, G["e2e_wav"], atol=FP32_ATOL, rtol=FP32_RTOL)


GS = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_spk.npz"))


@pytest.fixture(scope="module")
def spk_engine():
    from gonova_tts_amd.config import AcousticConfig
    w = make_acoustic_weights(seed=0, cfg=AcousticConfig(speaker_embed_dim=64))
    e = HipEngine(DEV, vocoder_dtype="f32", acoustic_dtype="f32")
    e.load_weights(acoustic=w, vocoder=make_vocoder_weights(seed=0))
    return e, w


def test_speaker_embedding_matches_golden_batched(spk_engine):
    """Speaker-embedding conditioning (HF:1192-1196): two utterances
    with different embeddings in one ragged batch against the transformers goldens
    (tests/golden/make_spk_golden.py); without embeddings the projection is skipped (HF)."""
    eng, w = spk_engine
    assert eng.speaker_dim == 64
    tags = ["spk_a", "spk_b"]
    ids_list = [GS[f"{t}_ids"] for t in tags]
    B, N = len(tags), max(len(x) for x in ids_list)
    tok = np.zeros((B, N), np.int32)
    for b, x in enumerate(ids_list):
        tok[b, :len(x)] = x
    lens = torch.tensor([len(x) for x in ids_list], dtype=torch.int32)
    emb = np.stack([GS[f"{t}_emb"] for t in tags])
    mel, mel_lens, dur = eng.acoustic(torch.from_numpy(tok).to(DEV), lens, 160, return_durations=True,
                                      speaker_embedding=torch.from_numpy(emb))
    mel0, mel_lens0 = eng.acoustic(torch.from_numpy(tok).to(DEV), lens, 160)
    for b, t in enumerate(tags):
        np.testing.assert_array_equal(dur[b, :len(ids_list[b])].cpu().numpy(), GS[f"{t}_dur"])
        L = int(mel_lens[b])
        assert L == GS[f"{t}_mel"].shape[0]
        np.testing.assert_allclose(mel[b, :L].cpu().numpy(), GS[f"{t}_mel"], atol=FP32_ATOL, rtol=FP32_RTOL)
        L0 = int(mel_lens0[b])
        assert L0 == GS[f"{t}_mel_nospk"].shape[0]
        np.testing.assert_allclose(mel0[b, :L0].cpu().numpy(), GS[f"{t}_mel_nospk"], atol=FP32_ATOL, rtol=FP32_RTOL)


def test_speaker_embedding_file_through_generate(spk_engine, tmp_path):
    """model.generate(text, audio_prompt_path=<stored embedding>) honours the voice (the
    reference's voice_id -> audio_prompt_path, server.py:127-138); scaling the embedding does
    not change the output (it is L2-normalised), a different voice does."""
    from gonova_tts_amd.config import AcousticConfig, VocoderConfig
    from gonova_tts_amd.model import GonovaTTS
    eng, w = spk_engine
    m = GonovaTTS(eng, AcousticConfig(speaker_embed_dim=64), VocoderConfig())
    np.save(tmp_path / "v1.npy", GS["spk_a_emb"])
    np.save(tmp_path / "v1x3.npy", 3.0 * GS["spk_a_emb"])
    np.save(tmp_path / "v2.npy", GS["spk_b_emb"])
    a = m.generate("Hello there.", audio_prompt_path=str(tmp_path / "v1.npy")).cpu().numpy()
    a3 = m.generate("Hello there.", audio_prompt_path=str(tmp_path / "v1x3.npy")).cpu().numpy()
    b = m.generate("Hello there.", audio_prompt_path=str(tmp_path / "v2.npy")).cpu().numpy()
    n = m.generate("Hello there.", audio_prompt_path="/nonexistent/voice.wav").cpu().numpy()
    assert a.shape == a3.shape and np.abs(a - a3).max() <= 1e-5 * max(1.0, np.abs(a).max())
    assert a.shape != b.shape or not np.allclose(a, b)
    assert n.size > 0


def test_generate_batch_mixed_voices_equals_single(spk_engine, tmp_path):
    """generate_batch with per-sentence voices (some None) == one generate call per sentence."""
    from gonova_tts_amd.config import AcousticConfig, VocoderConfig
    from gonova_tts_amd.model import GonovaTTS
    eng, _ = spk_engine
    m = GonovaTTS(eng, AcousticConfig(speaker_embed_dim=64), VocoderConfig())
    texts = ["Good morning.", "A second, longer sentence here.", "Third."]
    embs = [GS["spk_a_emb"], None, GS["spk_b_emb"]]
    batch = m.generate_batch(texts, speaker_embeddings=embs)
    for t, e, got in zip(texts, embs, batch):
        path = None
        if e is not None:
            path = str(tmp_path / f"{abs(hash(t))}.npy")
            np.save(path, e)
        ref = m.generate(t, audio_prompt_path=path).squeeze().cpu().numpy()
        assert got.shape == ref.shape
        assert np.abs(got - ref).max() <= 1e-4


@pytest.mark.parametrize("dtype", ["bf16", "f16", "f32"])
def test_fused_rel_attention_matches_unfused_and_oracle(aw, dtype, switch):
    """The fused relative-position attention (attention.hip: the 16-bit kernel for 16-bit
    stacks, the fp32 kernel for fp32 stacks -- the exact-duration encoder of every dtype here)
    against the four-launch path (TTS_REL_ATTN=0) and the oracle, on a ragged batch whose
    lengths cross the 64-query / 32-key tile edges (durations forced: predicted durations
    may legitimately round differently between two 16-bit paths).  fp32: both paths multiply
    in exact f32 and differ only in summation order and the online softmax's rescaling."""
    eng = engine(dtype, aw)
    rng = np.random.default_rng(11)
    ids_list = [rng.integers(1, 78, size=n) for n in (40, 1, 17, 33)]
    durs = [np.full(len(x), 5) for x in ids_list]
    switch("TTS_REL_ATTN", 1)
    fused, lf, _ = run(eng, ids_list, t_cap=200, durations=durs)
    switch("TTS_REL_ATTN", 0)
    unfused, lu, _ = run(eng, ids_list, t_cap=200, durations=durs)
    tol = {"bf16": 2.5e-2, "f16": 5e-3, "f32": 1e-5}[dtype]
    for b, ids in enumerate(ids_list):
        L = int(lf[b])
        assert L == int(lu[b]) == len(ids) * 5
        assert rel_rms(fused[b, :L], unfused[b, :L]) <= tol, (b, rel_rms(fused[b, :L], unfused[b, :L]))
        ref = acoustic_forward(ids, aw, durations=durs[b])
        if dtype == "f32":  # the fp32 golden tolerance (module docstring)
            np.testing.assert_allclose(fused[b, :L], ref["mel"], atol=FP32_ATOL, rtol=FP32_RTOL)
        else:
            check(f"acoustic {dtype} fused attention b={b} ({len(ids)} tokens)", fused[b, :L], ref["mel"],
                  kind="ac_" + dtype)
        assert np.all(fused[b, L:] == 0)


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_attention_key_groups_match(aw, dtype, switch):
    """The 16-bit attention with the block's keys split over two groups of 4 waves
    (TTS_ATTN_KSPLIT=1, merged through LDS) against the one-group kernel and the oracle: ragged
    lengths where the second group is empty (1, 17 tokens x 5 frames <= 96 keys), partial and
    full (utterances up to 500 frames)."""
    eng = engine(dtype, aw)
    rng = np.random.default_rng(13)
    ids_list = [rng.integers(1, 78, size=n) for n in (100, 1, 17, 33, 64)]
    durs = [np.full(len(x), 5) for x in ids_list]
    one, l1, _ = run(eng, ids_list, t_cap=500, durations=durs)
    switch("TTS_ATTN_KSPLIT", 1)
    two, l2, _ = run(eng, ids_list, t_cap=500, durations=durs)
    tol = {"bf16": 2.5e-2, "f16": 5e-3}[dtype]
    for b, ids in enumerate(ids_list):
        L = int(l1[b])
        assert L == int(l2[b]) == len(ids) * 5
        assert np.isfinite(two[b]).all()
        assert rel_rms(two[b, :L], one[b, :L]) <= tol, (b, rel_rms(two[b, :L], one[b, :L]))
        ref = acoustic_forward(ids, aw, durations=durs[b])
        check(f"acoustic {dtype} two key groups b={b} ({len(ids)} tokens)", two[b, :L], ref["mel"],
              kind="ac_" + dtype)
        assert np.all(two[b, L:] == 0)


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_short_row_tiles_bit_identical(aw, dtype, switch):
    """conv_xres picks 64-row tiles where 128-row tiles would leave much of each utterance's
    last tile empty (the encoder's short token rows), and 96-row tiles where they balance a small
    grid (the batch-8 decoder's 384-channel layers).  The channel group, and so the K order
    of the accumulation, is the same for every tile height, so the mel matches the 128-row
    run bit for bit (ragged batch, lengths across 64-row edges, durations forced) -- the
    property the chunked vocoder's bit-exactness rests on.  The narrow 64 x 64 tiles picked
    for under-filled grids (this batch of 4 picks them everywhere eligible) keep the same K
    order too: forced on, forced off and automatic all agree bit for bit."""
    eng = engine(dtype, aw)
    rng = np.random.default_rng(12)
    ids_list = [rng.integers(1, 78, size=n) for n in (144, 1, 65, 70)]
    durs = [np.full(len(x), 3) for x in ids_list]
    switch("TTS_XRES_NARROW", 0)   # 128-channel tiles: the tile-height pair
    switch("TTS_XRES_NT", 4)
    big, lb, _ = run(eng, ids_list, t_cap=432, durations=durs)
    switch("TTS_XRES_NT", 2)
    small, ls, _ = run(eng, ids_list, t_cap=432, durations=durs)
    switch("TTS_XRES_NT", 3)       # 96-row tiles (the 1- and 3-tap DMA forms; others keep their auto height)
    mid, lm, _ = run(eng, ids_list, t_cap=432, durations=durs)
    switch("TTS_XRES_NT", None)
    switch("TTS_XRES_NARROW", 1)   # 64 x 64 tiles wherever eligible
    narrow, ln, _ = run(eng, ids_list, t_cap=432, durations=durs)
    switch("TTS_XRES_NARROW", None)
    auto, la, _ = run(eng, ids_list, t_cap=432, durations=durs)
    for b, ids in enumerate(ids_list):
        L = int(la[b])
        assert int(lb[b]) == L == int(ls[b]) == int(ln[b]) == int(lm[b]) == len(ids) * 3
        assert np.array_equal(auto[b], big[b]) and np.array_equal(small[b], big[b]), b
        assert np.array_equal(mid[b], big[b]), b
        assert np.array_equal(narrow[b], big[b]), b
        ref = acoustic_forward(ids, aw, durations=durs[b])
        check(f"acoustic {dtype} short row tiles b={b}", auto[b, :L], ref["mel"], kind="ac_" + dtype)


@pytest.mark.parametrize("dtype,precision", [("bf16", "exact"), ("f16", "exact"), ("bf16", "fast")])
def test_fused_layernorm_bit_identical(aw, dtype, precision, switch):
    """The post-LNs applied inside the GEMM launches (the row tile's last M block normalises its
    rows: conv_xres for 16-bit stacks, the one-slice split GEMM for the exact encoder and its
    predictors, LayerNorm + Linear(C -> 1) for each predictor's last layer) give the same bits as
    the separate LayerNorm launches (TTS_LN_FUSE=0): predicted durations, frame counts and mel,
    on the default rule (grids of >= 512 blocks) and forced on every eligible launch (7), twice
    each.  A ragged batch whose lengths cross 64- and 128-row tile edges, and the C3 shape."""
    eng = engine(dtype, aw) if precision == "exact" else HipEngine(DEV, vocoder_dtype="f32", acoustic_dtype=dtype,
                                                                    encoder_precision="fast")
    if precision == "fast":
        eng.load_weights(acoustic=aw)
    rng = np.random.default_rng(41)
    cases = [[rng.integers(1, 78, size=n) for n in (144, 1, 65, 70, 127, 129, 9, 33)],
             [rng.integers(1, 78, size=144) for _ in range(32)]]
    for ids_list in cases:
        switch("TTS_LN_FUSE", 0)
        m0, l0, d0 = run(eng, ids_list, t_cap=8 * 144)
        for mode in (None, 7):  # default (grids of >= 512 blocks), every eligible launch
            switch("TTS_LN_FUSE", mode)
            for _ in range(2):  # (the hand-off must not depend on timing)
                m1, l1, d1 = run(eng, ids_list, t_cap=8 * 144)
                assert np.array_equal(d0, d1) and np.array_equal(l0, l1), mode
                assert np.array_equal(m0, m1), mode
    # (every oracle test of this file runs the fused default path)
    if precision == "fast":
        eng.close()


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_dma_staged_ffn_bit_identical(aw, dtype, switch):
    """The LDS-DMA form of conv_xres (X tiles copied global -> LDS one or two channel groups ahead,
    swizzled 128-byte rows) for the FFN convs and the 1-tap projections gives the register-staged
    kernel's bits (TTS_XRES_DMA=2; =3: the 1-tap projections register-staged), at both tile
    heights, on a ragged batch with predicted durations (narrow tiles off, so every eligible launch
    takes the 128-channel kernel); and the mel stays within the oracle tolerance."""
    eng = engine(dtype, aw)
    rng = np.random.default_rng(43)
    ids_list = [rng.integers(1, 78, size=n) for n in (144, 1, 65, 70, 127, 129, 9, 33)]
    outs = {}
    switch("TTS_XRES_NARROW", 0)
    for dma in (None, 3, 2):
        for nt in (2, 4):
            switch("TTS_XRES_DMA", dma)
            switch("TTS_XRES_NT", nt)
            outs[(dma, nt)] = run(eng, ids_list, t_cap=8 * 144)
    switch("TTS_XRES_NT", None)
    switch("TTS_XRES_DMA", None)
    switch("TTS_XRES_NARROW", None)
    ref_m, ref_l, ref_d = outs[(2, 4)]
    for k, (m, l, d) in outs.items():
        assert np.array_equal(d, ref_d) and np.array_equal(l, ref_l), k
        assert np.array_equal(m, ref_m), k
    durs = [ref_d[b, :len(x)] for b, x in enumerate(ids_list)]
    forced, fl, _ = run(eng, ids_list, t_cap=8 * 144, durations=durs)
    for b in (0, 4):
        L = int(fl[b])
        ref = acoustic_forward(ids_list[b], aw, durations=durs[b])
        check(f"acoustic {dtype} DMA-staged FFN b={b}", forced[b, :L], ref["mel"], kind="ac_" + dtype)


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_split_tile_height_bit_identical(aw, dtype, switch):
    """The split-precision GEMMs' 32-row tiles (small grids: the batch-8 exact encoder) give the
    64-row tiles' bits (TTS_SPLIT_NT1=0) and those of 32-row (=1) and 128-row (=4, the batch-32
    form) tiles everywhere, with the
    post-LNs fused in every eligible launch as well (TTS_LN_FUSE=7: the tail on 32-row tiles), on
    a ragged batch-8 forward with predicted durations."""
    eng = engine(dtype, aw)
    rng = np.random.default_rng(45)
    ids_list = [rng.integers(1, 78, size=n) for n in (144, 1, 65, 70, 127, 129, 9, 33)]
    outs = {}
    for nt1 in (0, None, 1, 4):
        for ln in (None, 7):
            switch("TTS_SPLIT_NT1", nt1)
            switch("TTS_LN_FUSE", ln)
            outs[(nt1, ln)] = run(eng, ids_list, t_cap=8 * 144)
    switch("TTS_SPLIT_NT1", None)
    switch("TTS_LN_FUSE", None)
    ref_m, ref_l, ref_d = outs[(0, None)]
    for k, (m, l, d) in outs.items():
        assert np.array_equal(d, ref_d) and np.array_equal(l, ref_l), k
        assert np.array_equal(m, ref_m), k


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_xcd_ordered_xres_grid_bit_identical(aw, dtype, switch):
    """conv_xres launched on a 1-D grid whose blocks are renumbered so that each XCD (blockIdx
    mod 8) walks a contiguous run of M blocks over the same X rows (TTS_XRES_ORDER=1: the
    multi-M-block launches; =2: every launch) gives the 3-D grid's bits, fused post-LN counters
    included, on a ragged batch with predicted durations at both tile heights."""
    eng = engine(dtype, aw)
    rng = np.random.default_rng(46)
    ids_list = [rng.integers(1, 78, size=n) for n in (144, 1, 65, 70, 127, 129, 9, 33)]
    outs = {}
    for order in (0, 1, 2):
        for nt in (None, 2):
            switch("TTS_XRES_ORDER", order)
            switch("TTS_XRES_NT", nt)
            outs[(order, nt)] = run(eng, ids_list, t_cap=8 * 144)
    switch("TTS_XRES_NT", None)
    switch("TTS_XRES_ORDER", None)
    ref_m, ref_l, ref_d = outs[(0, None)]
    for k, (m, l, d) in outs.items():
        assert np.array_equal(d, ref_d) and np.array_equal(l, ref_l), k
        assert np.array_equal(m, ref_m), k


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_split_whole_slice_staging_bit_identical(aw, dtype, switch):
    """Small split-precision GEMM grids (at most one block per CU: the batch-8 exact encoder and
    predictors) stage every channel group of their K slice at once; the quads and their MFMA order
    are those of the group-by-group form (TTS_SPLIT_WHOLE=0), so durations and mel match bit for
    bit on a ragged batch-8 forward with predicted durations."""
    eng = engine(dtype, aw)
    rng = np.random.default_rng(44)
    ids_list = [rng.integers(1, 78, size=n) for n in (144, 1, 65, 70, 127, 129, 9, 33)]
    switch("TTS_SPLIT_WHOLE", 0)
    m0, l0, d0 = run(eng, ids_list, t_cap=8 * 144)
    switch("TTS_SPLIT_WHOLE", None)
    m1, l1, d1 = run(eng, ids_list, t_cap=8 * 144)
    assert np.array_equal(d0, d1) and np.array_equal(l0, l1)
    assert np.array_equal(m0, m1)


def test_failed_reserve_leaves_a_usable_engine(aw):
    """A workspace reservation that runs out of device memory partway (advisor finding: the
    caps must never describe freed memory) raises, and the next small forward re-reserves
    and matches the result from before the failure bit for bit."""
    eng = HipEngine(DEV, vocoder_dtype="f32", acoustic_dtype="bf16")
    eng.load_weights(acoustic=aw)
    rng = np.random.default_rng(77)
    ids_list = [rng.integers(1, 78, size=n) for n in (30, 12)]
    durs = [np.full(len(x), 4) for x in ids_list]
    before, lb, _ = run(eng, ids_list, t_cap=120, durations=durs)
    with pytest.raises(RuntimeError):
        eng.reserve(512, 60000, 144)  # > 288 GB of workspace: some buffers allocate, then one fails
    after, la, _ = run(eng, ids_list, t_cap=120, durations=durs)
    assert np.array_equal(lb, la) and np.array_equal(before, after)
    eng.close()


def _oracle_log_durations(ids, aw):
    """fp32 oracle encoder + duration predictor only (HF:1171-1208), the log-durations that
    clamp(round(exp(x) - 1), 0) (HF:181-183) turns into integers."""
    from oracle.acoustic import conformer_stack, variance_predictor
    x = aw["encoder.embed.weight"][np.asarray(ids, np.int64)]
    x = conformer_stack(x, aw, "encoder.", 4, 2)
    return variance_predictor(x, aw, "duration_predictor.", 2)


def _margin(logd):
    """distance of the oracle's exp(x)-1 from the nearest .5 rounding boundary"""
    return np.abs((np.exp(logd.astype(np.float32)) - 1) % 1 - 0.5)


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_predicted_durations_exact_on_default_path(aw, dtype):
    """The default 16-bit acoustic path (encoder_precision="exact": encoder, speaker projection and
    variance predictors in fp32 with three-f16-MFMA GEMMs, conv_split.hip, and the split-precision
    fused attention, attention.hip) predicts integer
    durations equal to the fp32 oracle's for every token whose oracle exp(x)-1 is more than 1e-3
    from a .5 boundary -- the same carve-out as the fp32 path above.  C3's token distribution
    (32 x 144 ids U[1,77], 4,608 tokens), the two transformers golden utterances and a ragged tail."""
    eng = engine(dtype, aw)
    rng = np.random.default_rng(2000)
    ids_list = [rng.integers(1, 78, size=144) for _ in range(32)]
    ids_list += [G["ac_a_ids"], G["ac_b_ids"], rng.integers(1, 78, size=7), rng.integers(1, 78, size=1)]
    _, _, dur = run(eng, ids_list, t_cap=12 * 144)
    bad = total = carved = 0
    for b, ids in enumerate(ids_list):
        logd = _oracle_log_durations(ids, aw)
        ref = np.maximum(np.round(np.exp(logd.astype(np.float32)) - np.float32(1)), 0).astype(np.int64)
        ok = _margin(logd) > 1e-3
        got = dur[b, :len(ids)]
        bad += int((got[ok] != ref[ok]).sum())
        total += int(ok.sum())
        carved += int((~ok).sum())
    print(f"[parity] durations {dtype} exact-encoder: {bad} of {total} tokens differ "
          f"({carved} within 1e-3 of a .5 boundary not compared)")
    assert bad == 0
    for tag in ("ac_a", "ac_b"):  # the transformers goldens themselves
        b = len(ids_list) - 4 + (tag == "ac_b")
        np.testing.assert_array_equal(dur[b, :len(G[f"{tag}_ids"])], G[f"{tag}_dur"])


def test_predicted_durations_bf16_mel_matches_oracle(aw):
    """Predicted (not forced) durations on the default bf16 path end to end: the frame counts
    equal the oracle's, so the mel is comparable frame for frame (tests/parity.py ac_bf16)."""
    eng = engine("bf16", aw)
    rng = np.random.default_rng(31)
    ids_list = [rng.integers(1, 78, size=n) for n in (48, 21)]
    mel, mel_lens, dur = run(eng, ids_list, t_cap=12 * 48)
    for b, ids in enumerate(ids_list):
        ref = acoustic_forward(ids, aw)
        np.testing.assert_array_equal(dur[b, :len(ids)], ref["durations"])
        L = int(mel_lens[b])
        assert L == ref["mel"].shape[0]
        check(f"acoustic bf16 predicted-dur b={b}", mel[b, :L], ref["mel"], kind="ac_bf16")
        assert np.all(mel[b, L:] == 0)


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_batched_variance_predictors_bit_identical(aw, dtype, switch):
    """The variance predictors' first convs as one GEMM and their first LayerNorms as one grouped
    launch (acoustic.cpp batch_predictors / predict_batched, fp32 encoder activations) against the
    per-predictor launches (TTS_VP_BATCH=0): the same durations and mel bit for bit, with predicted
    durations (three predictors) and given ones (pitch and energy only), on a ragged batch."""
    eng = engine(dtype, aw)
    rng = np.random.default_rng(43)
    ids_list = [rng.integers(1, 78, size=n) for n in (57, 1, 30, 44)]
    durs = [rng.integers(0, 9, size=len(x)) for x in ids_list]
    for d in (None, durs):
        switch("TTS_VP_BATCH", 0)
        m0, l0, d0 = run(eng, ids_list, t_cap=12 * 57, durations=d)
        switch("TTS_VP_BATCH", None)
        m1, l1, d1 = run(eng, ids_list, t_cap=12 * 57, durations=d)
        assert np.array_equal(l1, l0) and np.array_equal(d1, d0), d is None
        assert np.array_equal(m1, m0), d is None


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_decoder_extent_trim_bit_identical(aw, dtype, switch):
    """With predicted durations the decoder runs at the longest utterance's frame count, read back
    after the variance adaptor, not at the caller's budget t_cap (acoustic.cpp forward,
    TTS_DEC_TRIM): the same mel, lengths and durations bit for bit as the decoder at t_cap, for
    a ragged batch at three budgets (12, 7 frames per token, and one that cuts the longest
    utterance short), with the output zero past each length."""
    eng = engine(dtype, aw)
    rng = np.random.default_rng(41)
    ids_list = [rng.integers(1, 78, size=n) for n in (60, 1, 33, 47, 12)]
    for t_cap in (12 * 60, 7 * 60, 200):
        switch("TTS_DEC_TRIM", 0)
        m0, l0, d0 = run(eng, ids_list, t_cap=t_cap)
        switch("TTS_DEC_TRIM", 1)
        m1, l1, d1 = run(eng, ids_list, t_cap=t_cap)
        assert m1.shape == m0.shape == (len(ids_list), t_cap, 80)
        assert np.array_equal(l1, l0) and np.array_equal(d1, d0), t_cap
        assert np.array_equal(m1, m0), t_cap
        for b in range(len(ids_list)):
            assert np.all(m1[b, int(l1[b]):] == 0)
        assert int(l1.max()) <= t_cap


def test_fast_encoder_precision_bounded():
    """encoder_precision="fast" (the whole acoustic model in bf16) stays available: its durations
    may round differently near .5 (measured 131 of 4,608 C3 tokens, all within 0.1 of a boundary);
    bounded here at 5 % of tokens, none off by more than one frame."""
    aw = make_acoustic_weights(seed=0)
    e = HipEngine(DEV, vocoder_dtype="f32", acoustic_dtype="bf16", encoder_precision="fast")
    e.load_weights(acoustic=aw)
    rng = np.random.default_rng(2000)
    ids_list = [rng.integers(1, 78, size=144) for _ in range(8)]
    _, _, dur = run(e, ids_list, t_cap=12 * 144)
    diff = np.concatenate([dur[b, :144] - np.maximum(np.round(np.exp(
        _oracle_log_durations(ids, aw).astype(np.float32)) - 1), 0) for b, ids in enumerate(ids_list)])
    print(f"[parity] durations bf16 fast-encoder: {int((diff != 0).sum())} of {diff.size} tokens differ")
    assert (diff != 0).mean() < 0.05 and np.abs(diff).max() <= 1
    e.close()


def test_range_guard_falls_back_to_fp32_encoder(aw):
    """Range guard of the exact encoder (include/tts_hip.h, ABI 4).  The split-precision GEMMs hold
    each fp32 operand as f16 halves, so an activation past 65504 would turn into inf.  Layer 0's
    macaron FFN up-projection is scaled by 2e4 (weights up to ~3,000, inside the finalize check)
    so its ReLU output reaches ~7.5e4: the forward sets the range word, the same forward on the
    fp32 MFMA encoder (TTS_ENCODER_F32) does not and matches the fp32 oracle (durations exact
    outside the .5 carve-out, bf16 mel through parity.py), GonovaTTS reruns the batch by itself
    (one RuntimeWarning, range_fallbacks == 1, finite audio), and the seeded weights never trip it."""
    from gonova_tts_amd.config import AcousticConfig, VocoderConfig
    from gonova_tts_amd.model import GonovaTTS
    ids_list = [np.random.default_rng(5).integers(1, 78, size=n) for n in (40, 23)]
    B, N = len(ids_list), 40
    tok = np.zeros((B, N), np.int32)
    for b, x in enumerate(ids_list):
        tok[b, :len(x)] = x
    lens = np.array([len(x) for x in ids_list], np.int32)
    tok_d, lens_d = torch.from_numpy(tok).to(DEV), torch.from_numpy(lens).to(DEV)
    # seeded weights: the word stays 0
    *_, rw = engine("bf16", aw).acoustic(tok_d, lens_d, 12 * N, return_range=True)
    assert int(rw.item()) == 0
    k = "encoder.conformer_layers.0.feed_forward_macaron.conv1.weight"
    aw2 = dict(aw)
    aw2[k] = aw[k] * 20000.0
    e = HipEngine(DEV, vocoder_dtype="f16", acoustic_dtype="bf16")
    e.load_weights(acoustic=aw2, vocoder=make_vocoder_weights(seed=0))
    *_, rw = e.acoustic(tok_d, lens_d, 12 * N, return_range=True)
    assert int(rw.item()) == 1
    with e.encoder_f32():
        mel, mel_lens, dur, rw = e.acoustic(tok_d, lens_d, 12 * N, return_durations=True, return_range=True)
    assert int(rw.item()) == 0
    mel, mel_lens, dur = mel.cpu().numpy(), mel_lens.cpu().numpy(), dur.cpu().numpy()
    for b, ids in enumerate(ids_list):
        ref = acoustic_forward(ids, aw2)
        logd = _oracle_log_durations(ids, aw2)
        ok = _margin(logd) > 1e-3
        np.testing.assert_array_equal(dur[b, :len(ids)][ok], ref["durations"][ok])
        if np.array_equal(dur[b, :len(ids)], ref["durations"]):
            L = int(mel_lens[b])
            check(f"acoustic bf16 range-guard fp32 encoder b={b}", mel[b, :L], ref["mel"], kind="ac_bf16")
    m = GonovaTTS(e, AcousticConfig(), VocoderConfig())
    with pytest.warns(RuntimeWarning, match="f16 range"):
        wav, wav_lens = m.synthesize_tokens(tok, lens)
    assert m.range_fallbacks == 1
    w = wav.cpu().numpy()
    assert np.isfinite(w).all() and list(wav_lens) == [int(x) * 256 for x in mel_lens]
    # the encoder is back on the split path afterwards: the next forward trips the word again
    *_, rw = e.acoustic(tok_d, lens_d, 12 * N, return_range=True)
    assert int(rw.item()) == 1
    # the sharded path (dist.ShardedSynthesis, one rank, given durations, host_lens=False: no host
    # read inside synthesize_tokens): the word is read with the lengths at the run's own sync and the
    # tripped bucket is synthesized again on the fp32 encoder -- finite audio, not inf
    from gonova_tts_amd.dist import ShardedSynthesis

    def synth(t, l):
        d = np.where(np.arange(t.shape[1])[None, :] < l[:, None], 6, 0).astype(np.int32)
        return m.synthesize_tokens(t, l, durations=d, host_lens=False)

    with pytest.warns(RuntimeWarning, match="f16 range"):
        out = ShardedSynthesis(synth, torch.device(DEV), bucket=4).run(tok, lens)
    assert m.range_fallbacks == 2
    for b in range(B):
        assert out[b].shape == (int(lens[b]) * 6 * 256,) and np.isfinite(out[b]).all(), b
    # streaming with predicted durations: the first pass trips, the fallback runs on the
    # fp32 encoder, and with a 64-frame first cap (the durations need 172 / 103 frames) the second,
    # longer pass must stay on the fp32 encoder too
    m.FRAMES_PER_TOKEN_CAP = 1
    with pytest.warns(RuntimeWarning, match="f16 range"):
        chunks = list(m.stream_tokens(tok, lens, chunk_frames=64))
    assert m.range_fallbacks == 3
    assert len(chunks) == 3  # 172 frames in 64-frame chunks: the second pass ran
    for c0, wav, valid in chunks:
        assert np.isfinite(wav.cpu().numpy()).all(), c0
    e.close()


def test_fp32_attention_key_chunks(aw, switch):
    """fp32 attention in key chunks merged by a second launch (attention.hip rel_attn_f32_kernel /
    rel_attn_merge_kernel, TTS_ATTN_F32_KC, >= 32 keys): an utterance whose stacks fit one chunk is
    bit-identical to the one-pass kernel (its merge is x * 2^0 then the same O / l); a longer one
    differs only by the merge's summation order (2e-6 relative bound here), and a 426-frame
    utterance (C1's sentence: several decoder chunks) matches the oracle at the fp32 bar."""
    eng = engine("f32", aw)
    rng = np.random.default_rng(23)
    ids_list = [rng.integers(1, 78, size=n) for n in (71, 5, 30)]
    durs = [np.full(len(x), 6, np.int32) for x in ids_list]  # 426, 30, 180 frames
    t_cap = 426
    switch("TTS_ATTN_F32_KC", 0)
    m0, l0, _ = run(eng, ids_list, t_cap=t_cap, durations=durs)
    switch("TTS_ATTN_F32_KC", None)  # the default chunk
    m1, l1, _ = run(eng, ids_list, t_cap=t_cap, durations=durs)
    assert np.array_equal(l0, l1) and list(l1) == [426, 30, 180]
    assert np.array_equal(m1[1, :30], m0[1, :30])  # one chunk in both stacks (<= 32 keys)
    for b in (0, 2):
        L = int(l1[b])
        err = np.abs(m1[b, :L] - m0[b, :L]).max() / np.abs(m0[b, :L]).max()
        assert err < 2e-6, (b, err)
    ref = acoustic_forward(ids_list[0], aw, durations=durs[0])
    np.testing.assert_allclose(m1[0, :426], ref["mel"], atol=FP32_ATOL, rtol=FP32_RTOL)


def test_fp32_model_split_encoder_matches_fp32_mfma_encoder(aw, switch):
    """An fp32 model's encoder side on split-precision GEMMs and attention (TTS_ENCODER_EXACT with
    acoustic_dtype f32, round 6) against the same model with every layer on fp32 MFMA
    (TTS_F32_ENC_SPLIT=0 at finalize): identical predicted durations and frame counts on a
    ragged batch, mel within the fp32 bar; the range guard is on for the fp32 model, and a
    scaled layer trips it and falls back to the fp32 encoder (no inf in the mel)."""
    rng = np.random.default_rng(31)
    ids_list = [rng.integers(1, 78, size=n) for n in (71, 9, 40)]
    switch("TTS_F32_ENC_SPLIT", 0)
    e0 = HipEngine(DEV, vocoder_dtype="f32", acoustic_dtype="f32")
    e0.load_weights(acoustic=aw)
    switch("TTS_F32_ENC_SPLIT", None)
    e1 = HipEngine(DEV, vocoder_dtype="f32", acoustic_dtype="f32")
    e1.load_weights(acoustic=aw)
    assert e1.range_guard and not e0.range_guard
    m0, l0, d0 = run(e0, ids_list, t_cap=12 * 71)
    m1, l1, d1 = run(e1, ids_list, t_cap=12 * 71)
    assert np.array_equal(d0, d1) and np.array_equal(l0, l1)
    for b in range(len(ids_list)):
        L = int(l1[b])
        np.testing.assert_allclose(m1[b, :L], m0[b, :L], atol=FP32_ATOL, rtol=FP32_RTOL)
    e0.close()
    k = "encoder.conformer_layers.0.feed_forward_macaron.conv1.weight"
    aw2 = dict(aw)
    aw2[k] = aw[k] * 20000.0
    e2 = HipEngine(DEV, vocoder_dtype="f32", acoustic_dtype="f32")
    e2.load_weights(acoustic=aw2)
    B, N = len(ids_list), 71
    tok = np.zeros((B, N), np.int32)
    for b, x in enumerate(ids_list):
        tok[b, :len(x)] = x
    tok_d = torch.from_numpy(tok).to(DEV)
    lens_d = torch.tensor([len(x) for x in ids_list], dtype=torch.int32, device=DEV)
    *_, rw = e2.acoustic(tok_d, lens_d, 12 * N, return_range=True)
    assert int(rw.item()) == 1
    with e2.encoder_f32():
        mel, mel_lens, rw = e2.acoustic(tok_d, lens_d, 12 * N, return_range=True)
    assert int(rw.item()) == 0 and torch.isfinite(mel).all()
    e1.close()
    e2.close()


def test_predicted_duration_forward_captures_into_a_graph(aw):
    """with predicted durations and a loose budget the forward reads the frame counts back
    mid-call (TTS_DEC_TRIM); on a stream being captured into a HIP graph it skips that read and runs
    the decoder at the budget instead, so the capture succeeds, and the replay's mel and frame counts
    equal the eager (trimmed) forward's bit for bit."""
    eng = engine("bf16", aw)
    rng = np.random.default_rng(77)
    ids_list = [rng.integers(1, 78, size=n) for n in (30, 12, 21)]
    B, N = len(ids_list), 30
    tok = np.zeros((B, N), np.int32)
    for b, x in enumerate(ids_list):
        tok[b, :len(x)] = x
    tok_d = torch.from_numpy(tok).to(DEV)
    tl = torch.tensor([len(x) for x in ids_list], dtype=torch.int32, device=DEV)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        mel0, l0 = eng.acoustic(tok_d, tl, 12 * N, stream=s)  # eager: trimmed; reserves the workspace
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        mel1, l1 = eng.acoustic(tok_d, tl, 12 * N, stream=s)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(l0, l1)
    assert torch.equal(mel0, mel1)


@pytest.mark.parametrize("n_tok", [32, 33])
def test_fp32_decoder_ffn_down_with_and_without_pad_rows(aw, n_tok):
    """The fp32 decoder's FFN down-projections run split-precision on the packed split-K form, which
    needs pad rows after the longest utterance: the decoder's row stride keeps two (acoustic.cpp
    dec_pad), so 192 frames (a multiple of 32: stride 224) and 198 frames (stride 224) both take
    it, and both match the oracle at the fp32 bar (the postnet's 80-channel last conv, with its
    residual, on the packed form too)."""
    eng = engine("f32", aw)
    ids = np.random.default_rng(100 + n_tok).integers(1, 78, size=n_tok)
    d = np.full(n_tok, 6, np.int32)
    mel, mel_lens, _ = run(eng, [ids], t_cap=6 * n_tok, durations=[d])
    L = int(mel_lens[0])
    assert L == 6 * n_tok
    ref = acoustic_forward(ids, aw, durations=d)
    np.testing.assert_allclose(mel[0, :L], ref["mel"], atol=FP32_ATOL, rtol=FP32_RTOL)
