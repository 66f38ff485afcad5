"""Probe: how often do predicted integer durations (HF:181-183) of the HIP acoustic model
disagree with the fp32 oracle, per acoustic dtype; and what the encoder costs per dtype.

    python tools/dur_probe.py [--timing]

Prints one JSON line per measurement.  The oracle (test infrastructure) is used only as the
checker: its encoder + duration predictor give the reference log-durations.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from gonova_tts_amd.engine import HipEngine  # noqa: E402
from gonova_tts_amd.weights import make_acoustic_weights  # noqa: E402
from oracle.acoustic import conformer_stack, variance_predictor, durations_from_log  # noqa: E402


def oracle_logd(ids, aw):
    x = aw["encoder.embed.weight"][np.asarray(ids, np.int64)]
    x = conformer_stack(x, aw, "encoder.", 4, 2)
    return variance_predictor(x, aw, "duration_predictor.", 2)


def main():
    aw = make_acoustic_weights(0)
    rng = np.random.default_rng(2000)
    B, N = 32, 144
    tok = rng.integers(1, 78, size=(B, N)).astype(np.int32)
    lens = np.full(B, N, np.int32)
    t0 = time.time()
    ref_logd = np.stack([oracle_logd(tok[b], aw) for b in range(B)])
    ref_dur = np.stack([durations_from_log(ref_logd[b]) for b in range(B)])
    margin = np.abs((np.exp(ref_logd.astype(np.float32)) - 1) % 1 - 0.5)
    print(json.dumps({"oracle_s": round(time.time() - t0, 2), "mean_dur": float(ref_dur.mean()),
                      "frac_margin_lt_1e-3": float((margin < 1e-3).mean()),
                      "frac_margin_lt_1e-2": float((margin < 1e-2).mean()),
                      "frac_margin_lt_3e-2": float((margin < 3e-2).mean())}), flush=True)
    for dt, prec in (("f32", "exact"), ("f16", "exact"), ("bf16", "exact"), ("f16", "fast"), ("bf16", "fast")):
        eng = HipEngine("cuda:0", vocoder_dtype="f32", acoustic_dtype=dt, encoder_precision=prec)
        eng.load_weights(acoustic=aw)
        mel, ml, dur = eng.acoustic(torch.from_numpy(tok).cuda(), torch.from_numpy(lens), 12 * N,
                                    return_durations=True)
        torch.cuda.synchronize()
        d = dur.cpu().numpy()
        bad = d != ref_dur
        print(json.dumps({"dtype": dt, "encoder": prec, "mismatch_tokens": int(bad.sum()), "tokens": int(bad.size),
                          "utts_with_mismatch": int(bad.any(axis=1).sum()),
                          "max_margin_of_mismatch": float(margin[bad].max()) if bad.any() else None,
                          "median_margin_of_mismatch": float(np.median(margin[bad])) if bad.any() else None}),
              flush=True)
        if "--timing" in sys.argv:
            for Bt in (32, 8):
                for fr in (6, 1):
                    tk = torch.from_numpy(tok[:Bt]).cuda()
                    tl = torch.from_numpy(lens[:Bt])
                    dd = torch.full((Bt, N), fr, dtype=torch.int32, device="cuda")
                    for _ in range(3):
                        eng.acoustic(tk, tl, N * fr, durations=dd)
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    for _ in range(10):
                        eng.acoustic(tk, tl, N * fr, durations=dd)
                    torch.cuda.synchronize()
                    print(json.dumps({"dtype": dt, "encoder": prec, "B": Bt, "frames_per_token": fr,
                                      "acoustic_ms": round((time.perf_counter() - t) * 100, 3)}), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
