"""Measured error of the fp32 acoustic path against the transformers goldens and the oracle
(the numbers tests/test_acoustic_gpu.py's fp32 tolerances are derived from).

usage (GPU box): python3 tools/fp32_err_probe.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from gonova_tts_amd.engine import HipEngine
    from oracle.acoustic import acoustic_forward
    G = dict(np.load(os.path.join(ROOT, "tests", "golden", "golden_v1.npz")))
    from gonova_tts_amd.weights import make_acoustic_weights
    aw = make_acoustic_weights(seed=0)  # the tests' weights
    eng = HipEngine("cuda:0", acoustic_dtype="f32", vocoder_dtype="f32")
    eng.load_weights(acoustic=aw)

    def run(ids_list, t_cap):
        nonlocal eng
        B, N = len(ids_list), max(len(x) for x in ids_list)
        tok = np.zeros((B, N), np.int32)
        for b, x in enumerate(ids_list):
            tok[b, :len(x)] = x
        lens = torch.tensor([len(x) for x in ids_list], dtype=torch.int32)
        mel, ml, dur = eng.acoustic(torch.from_numpy(tok).cuda(), lens, t_cap, return_durations=True)
        torch.cuda.synchronize()
        return mel.cpu().numpy(), ml.cpu().numpy(), dur.cpu().numpy()

    for tag in ("ac_a", "ac_b"):
        ids = G[f"{tag}_ids"]
        mel, ml, dur = run([ids], 128)
        ref = G[f"{tag}_mel"]
        L = int(ml[0])
        d = np.abs(mel[0, :L] - ref)
        print(f"golden {tag}: max abs {d.max():.3e}, max rel {np.max(d / (np.abs(ref) + 1e-3)):.3e}, "
              f"rel-rms {np.sqrt(np.mean(d ** 2)) / np.sqrt(np.mean(ref ** 2)):.3e}")
    rng = np.random.default_rng(3)
    ids_list = [rng.integers(1, 78, size=n) for n in (20, 7, 33, 1)]
    mel, ml, dur = run(ids_list, 200)
    for b, ids in enumerate(ids_list):
        ref = acoustic_forward(ids, aw)
        if not np.array_equal(dur[b, :len(ids)], ref["durations"]):
            print(f"oracle b={b}: durations differ (rounding boundary)")
            continue
        L = int(ml[b])
        r = ref["mel"][:L]
        d = np.abs(mel[b, :L] - r)
        print(f"oracle b={b}: max abs {d.max():.3e}, max rel {np.max(d / (np.abs(r) + 1e-3)):.3e}, "
              f"rel-rms {np.sqrt(np.mean(d ** 2)) / np.sqrt(np.mean(r ** 2)):.3e}")
    eng.close()
    # end to end (tests/test_acoustic_gpu.py::test_end_to_end_fp32_matches_golden)
    from gonova_tts_amd.weights import make_vocoder_weights
    eng = HipEngine("cuda:0", acoustic_dtype="f32", vocoder_dtype="f32")
    eng.load_weights(acoustic=aw, vocoder=make_vocoder_weights(seed=0))
    mel, ml, _ = run([G["ac_a_ids"]], 64)
    L = int(ml[0])
    wav = eng.vocoder(torch.from_numpy(mel[:, :L].copy()).cuda()).cpu().numpy()[0]
    ref = G["e2e_wav"]
    d = np.abs(wav - ref)
    print(f"e2e wav: max abs {d.max():.3e}, rel-rms {np.sqrt(np.mean(d ** 2)) / np.sqrt(np.mean(ref ** 2)):.3e}, "
          f"max |d| - 1e-4 |ref| {np.max(d - 1e-4 * np.abs(ref)):.3e}")
    eng.close()


if __name__ == "__main__":
    main()
