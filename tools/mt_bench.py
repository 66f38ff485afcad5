"""Single-layer timing of the 16-bit acoustic GEMMs through the C-ABI (tts_op_conv1d -> conv_mt /
conv_xres / conv_gemm, whichever the library picks for the shape), at the C3 decoder's shapes.

usage (GPU box): python3 tools/mt_bench.py [layer ...]    (default: every layer below)
env: MT_B (utterances, 32), MT_T (rows per utterance, 864), MT_ITERS (50), TTS_MT_TILE / TTS_LIB as usual;
TTS_CONV_MT defaults to 1 here (the kernels under test; conv_xres needs the engine's packed weights).
Prints per layer: launches' mean time (hipEvents around MT_ITERS back-to-back launches), algorithmic
TFLOP/s, and the max relative error against a torch fp32 reference of the same conv on one utterance.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# name: (M, Cin, taps, act, residual, alpha)
LAYERS = {
    "ffn_up": (1536, 384, 3, 1, False, 1.0),
    "ffn_down": (384, 1536, 3, 0, True, 0.5),
    "qkv": (1152, 384, 1, 0, False, 1.0),
    "out_proj": (384, 384, 1, 0, True, 1.0),
    "pw1": (768, 384, 1, 0, False, 1.0),
    "postnet": (256, 256, 5, 2, False, 1.0),
}


def main():
    os.environ.setdefault("TTS_CONV_MT", "1")  # conv_mt / conv_tap (opt-in in the product)
    import torch
    from gonova_tts_amd.engine import TtsConvDesc, conv1d_op, load_library
    load_library()
    B, T = int(os.environ.get("MT_B", "32")), int(os.environ.get("MT_T", "864"))
    iters = int(os.environ.get("MT_ITERS", "50"))
    names = [a for a in sys.argv[1:] if a in LAYERS] or list(LAYERS)
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    for name in names:
        M, Cin, k, act, res, alpha = LAYERS[name]
        x = (torch.randn(B, T, Cin, generator=g) * 0.5).to(dev, torch.bfloat16)
        w = (torch.randn(M, k, Cin, generator=g) / (Cin * k) ** 0.5).to(dev, torch.bfloat16)
        bias = (torch.randn(M, generator=g) * 0.1).to(dev)
        r = (torch.randn(B, T, M, generator=g) * 0.5).to(dev, torch.bfloat16) if res else None
        y = torch.empty(B, T, M, device=dev, dtype=torch.bfloat16)
        lens = torch.full((B,), T, dtype=torch.int32, device=dev)
        d = TtsConvDesc()
        d.x, d.sxb, d.sxr, d.x_len, d.x_rows = x.data_ptr(), T * Cin, Cin, lens.data_ptr(), T
        d.w, d.swb, d.w_ld, d.bias = w.data_ptr(), 0, k * Cin, bias.data_ptr()
        d.y, d.syb, d.syr = y.data_ptr(), T * M, M
        d.r1, d.r2, d.srb, d.srr = (r.data_ptr() if res else None), None, T * M, M
        d.y_len, d.y_rows = lens.data_ptr(), T
        d.M, d.Cin, d.taps, d.dil, d.pad = M, Cin, k, 1, (k - 1) // 2
        d.in_slope, d.act_out, d.out_slope, d.alpha, d.out_scale = 1.0, act, 0.0, alpha, 1.0
        d.up_s, d.up_cout, d.up_p, d.up_len, d.B = 0, 0, 0, None, B
        for _ in range(3):
            conv1d_op("bf16", d)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            conv1d_op("bf16", d)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        tf = 2.0 * M * Cin * k * B * T / (us * 1e-6) / 1e12
        # torch fp32 reference on utterance 0
        xf = x[0].float().t()[None]                     # [1, Cin, T]
        wf = w.float().permute(0, 2, 1)                 # [M, Cin, k]
        ref = torch.nn.functional.conv1d(xf, wf, bias, padding=(k - 1) // 2)[0].t() * alpha
        if act == 1:
            ref = torch.relu(ref)
        elif act == 2:
            ref = torch.tanh(ref)
        if res:
            ref = ref.to(torch.bfloat16).float() + r[0].float()
        err = float(((y[0].float() - ref).abs().max() / ref.abs().max()).item())
        print(f"{name:9s} M={M:5d} K={Cin * k:5d} B={B} T={T}: {us:8.2f} us  {tf:7.1f} TF/s  max rel err {err:.2e}",
              flush=True)


if __name__ == "__main__":
    main()
