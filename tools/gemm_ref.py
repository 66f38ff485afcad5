"""Library-GEMM yardstick for the acoustic layers: torch.matmul (hipBLASLt) on the same operand
shapes as tools/mt_bench.py's layers, taken as plain GEMMs (a k = 3 conv as one GEMM over an
im2col'd K = 3 * Cin; the im2col itself is not timed).  Not on the product path: it says what
a tuned library kernel reaches on MI355X for M x N x K of these sizes.

usage (GPU box): python3 tools/gemm_ref.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch
    from mt_bench import LAYERS
    B, T = int(os.environ.get("MT_B", "32")), int(os.environ.get("MT_T", "864"))
    iters = int(os.environ.get("MT_ITERS", "50"))
    dev = torch.device("cuda:0")
    for name, (M, Cin, k, act, res, alpha) in LAYERS.items():
        a = torch.randn(B * T, k * Cin, device=dev, dtype=torch.bfloat16)
        w = torch.randn(k * Cin, M, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            y = a @ w
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            y = a @ w
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        tf = 2.0 * M * Cin * k * B * T / (us * 1e-6) / 1e12
        print(f"{name:9s} [{B * T} x {k * Cin}] @ [{k * Cin} x {M}] hipBLASLt: {us:8.2f} us {tf:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
