"""Run-to-run stability of the fused LayerNorm hand-offs (ln_rows.h): the batch-32 C3-shape
acoustic forward (exact encoder, bf16) repeated, its mel hashed each time, with the fused post-LNs
on (default, and TTS_LN_FUSE=7: every eligible launch) and off (TTS_LN_FUSE=0: separate reduce +
LayerNorm launches, the reference bits).  Build variants with -DTTS_SPLITK_FUSE=1 (the in-launch
split-K reduce) and -DTTS_LN_RELEASE=0/1 and run each under TTS_LIB=...; every hash of one build
must be the same, and equal to the TTS_LN_FUSE=0 one."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(reps=4):
    import torch
    from gonova_tts_amd.engine import HipEngine, switches
    from gonova_tts_amd.weights import make_acoustic_weights
    aw = make_acoustic_weights(seed=0, fixed_duration=6)
    g = torch.Generator(device="cpu").manual_seed(11)
    B, N = 32, 144
    e = HipEngine("cuda:0", vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=B, max_frames=6 * N, max_tokens=N)
    e.load_weights(acoustic=aw)
    tok = torch.randint(1, 78, (B, N), generator=g, dtype=torch.int32).cuda()
    tl = torch.randint(100, N + 1, (B,), generator=g, dtype=torch.int32).cuda()
    res = {}
    for name, sw in (("fuse_default", {}), ("fuse_all", {"TTS_LN_FUSE": 7}), ("unfused", {"TTS_LN_FUSE": 0})):
        hs = []
        with switches(**sw):
            for _ in range(reps):
                m, ml, d = e.acoustic(tok, tl, 6 * N, return_durations=True)
                torch.cuda.synchronize()
                hs.append(hashlib.sha256(m.cpu().numpy().tobytes() + d.cpu().numpy().tobytes()).hexdigest()[:12])
        res[name] = hs
        print(name, " ".join(hs), "stable" if len(set(hs)) == 1 else "VARIES")
    ref = res["unfused"][0]
    print("all equal to unfused:", all(h == ref for v in res.values() for h in v))
    e.close()


if __name__ == "__main__":
    main()
