"""Output fingerprint of the default paths (C2-shape fp16 vocoder on 4 x 862 frames, bf16 C3-shape
acoustic + vocoder on 4 x 144 tokens, batch-8 acoustic), for bit-identity checks between two
library builds: run once per build (TTS_LIB=...) and compare the printed digests."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from gonova_tts_amd.engine import HipEngine
    from gonova_tts_amd.weights import make_acoustic_weights, make_vocoder_weights
    vw, aw = make_vocoder_weights(seed=0), make_acoustic_weights(seed=0, fixed_duration=6)
    g = torch.Generator(device="cpu").manual_seed(7)
    out = {}
    e = HipEngine("cuda:0", vocoder_dtype="f16")
    e.load_weights(vocoder=vw)
    mel = torch.randn((4, 862, 80), generator=g).cuda()
    out["c2_f16"] = e.vocoder(mel).cpu().numpy()
    e.close()
    for B in (4, 8):
        e = HipEngine("cuda:0", vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=B, max_frames=864, max_tokens=144)
        e.load_weights(vocoder=vw, acoustic=aw)
        tok = torch.randint(1, 78, (B, 144), generator=g, dtype=torch.int32).cuda()
        tl = torch.full((B,), 144, dtype=torch.int32).cuda()
        m, ml = e.acoustic(tok, tl, 864)
        out[f"mel_b{B}"] = m.cpu().numpy()
        out[f"wav_b{B}"] = e.vocoder(m, ml).cpu().numpy()
        if B == 8:  # ragged lengths: the attention kernels' partial key steps and padding rows
            tl = torch.randint(29, 145, (B,), generator=g, dtype=torch.int32).cuda()
            m, ml = e.acoustic(tok, tl, 864)
            valid = torch.arange(m.shape[1], device=m.device)[None, :] < ml[:, None].long()
            out["mel_ragged_b8"] = torch.where(valid[..., None], m, torch.zeros_like(m)).cpu().numpy()
        e.close()
    # fp32 engine (C1's): one 71-token utterance, tokens -> mel -> waveform
    e = HipEngine("cuda:0", vocoder_dtype="f32", acoustic_dtype="f32", max_batch=1, max_frames=426, max_tokens=71)
    e.load_weights(vocoder=vw, acoustic=aw)
    tok = torch.randint(1, 78, (1, 71), generator=g, dtype=torch.int32).cuda()
    m, ml = e.acoustic(tok, torch.full((1,), 71, dtype=torch.int32).cuda(), 426)
    out["c1_f32_mel"] = m.cpu().numpy()
    out["c1_f32_wav"] = e.vocoder(m, ml).cpu().numpy()
    e.close()
    for k, v in out.items():
        print(k, v.shape, hashlib.sha256(v.tobytes()).hexdigest()[:16])


if __name__ == "__main__":
    main()
