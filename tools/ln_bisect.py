"""Diagnostic: acoustic outputs with the fused post-LN paths on (TTS_LN_FUSE modes 1-7) against the
separate launches (0), bit for bit and over repetitions (LNB_B32=1: the C3 shape; LNB_MODES, LNB_REPS)."""
import sys

import numpy as np
sys.path.insert(0, '.')

def main():
    import torch
    from gonova_tts_amd.engine import HipEngine, set_switch
    from gonova_tts_amd.weights import make_acoustic_weights
    aw = make_acoustic_weights(seed=0)
    rng = np.random.default_rng(41)
    import os
    ids_list = [rng.integers(1, 78, size=n) for n in (144, 1, 65, 70, 127, 129, 9, 33)]
    if os.environ.get("LNB_B32"):
        ids_list = [rng.integers(1, 78, size=144) for _ in range(32)]
    MODES = [int(x) for x in os.environ.get("LNB_MODES", "0 1 2 3 4 5 6").split()]
    REPS = int(os.environ.get("LNB_REPS", "1"))
    B = len(ids_list); N = 144
    tok = np.zeros((B, N), np.int32)
    for b, x in enumerate(ids_list): tok[b, :len(x)] = x
    lens = torch.tensor([len(x) for x in ids_list], dtype=torch.int32)
    for prec in ("exact", "fast"):
        e = HipEngine("cuda:0", vocoder_dtype="f32", acoustic_dtype="bf16", encoder_precision=prec)
        e.load_weights(acoustic=aw)
        res = {}
        for v in MODES:
            set_switch("TTS_LN_FUSE", v)
            for _ in range(REPS):
                mel, ml, dur = e.acoustic(torch.from_numpy(tok).cuda(), lens, 8 * 144, return_durations=True)
                torch.cuda.synchronize()
                r = (mel.cpu().numpy(), ml.cpu().numpy(), dur.cpu().numpy())
                if v in res and not (np.array_equal(res[v][2], r[2]) and np.array_equal(res[v][0], r[0])):
                    print(prec, "mode", v, "NOT REPRODUCIBLE across repetitions", flush=True)
                res[v] = r
        for v in MODES[1:]:
            m0, l0, d0 = res[0]; m1, l1, d1 = res[v]
            print(prec, "mode", v, "dur eq", np.array_equal(d0, d1), "mel eq", np.array_equal(m0, m1) if np.array_equal(l0, l1) else "len differ",
                  "maxdiff", float(np.abs(m0 - m1).max()) if m0.shape == m1.shape else None, flush=True)
        e.close()


if __name__ == "__main__":
    main()
