"""bench.py — headline benchmark of the MI355X TTS engine (one JSON line on rank 0).

Workload (BASELINE.json configs[1], the config the metric is quoted on that fits one
GPU): HiFi-GAN V1 vocoder, batch 32 x 862 mel frames (10.008 s @ 22,050 Hz, 220,672
samples per utterance), fp16 activations / fp32 accumulation, synthetic mel ~ N(0,1)
already resident in HBM, deterministic seeded weights (no checkpoint offline).
A "step" = one vocoder forward over the batch.  `--workload full` runs configs[2]
(tokens -> acoustic -> vocoder, bf16 acoustic) instead.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
utterances are independent, so every rank runs its own batch-32 shard with no
data-path collective (weak scaling); rank timing is bracketed by barriers and the
max over ranks is reported.  value = samples of all ranks / max time.

Also reported: `roofline` for the dominant kernel family (the implicit-GEMM conv,
timed live with hipEvents around each launch on its stream) and `cpu_baseline`
(the NumPy oracle on the host cores, bounded sample, rank 0 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SR = 22050
METRIC = "audio samples/sec/GPU + real-time factor, batch-32 10s utterances @22.05kHz"
MFMA_PEAK_TFLOPS = {"f16": 2500.0, "bf16": 2500.0, "f32": 157.3}  # dense, MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--frames", type=int, default=862)
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--workload", default="vocoder", choices=["vocoder", "full"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=862, help="frames in the CPU-baseline sample")
    return ap.parse_args()


def cpu_baseline(frames: int):
    """NumPy fp32 oracle (oracle/vocoder.py) on one utterance of `frames` frames."""
    from gonova_tts_amd.weights import make_vocoder_weights
    from oracle.vocoder import vocoder_forward
    w = make_vocoder_weights(seed=0)
    mel = np.random.default_rng(0).standard_normal((frames, 80)).astype(np.float32)
    vocoder_forward(mel[:8], w)  # warm BLAS
    t = time.perf_counter()
    wav = vocoder_forward(mel, w)
    dt = time.perf_counter() - t
    threads = os.environ.get("OMP_NUM_THREADS") or os.environ.get("OPENBLAS_NUM_THREADS")
    cores = int(threads) if threads else (os.cpu_count() or 1)
    return {"value": len(wav) / dt, "unit": "samples/s", "cores": cores, "kind": "port",
            "sample": f"1 utterance x {frames} frames ({len(wav) / SR:.2f} s audio), NumPy fp32 oracle, "
                      f"{dt:.1f} s wall"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from gonova_tts_amd.engine import HipEngine
    from gonova_tts_amd.weights import make_vocoder_weights
    from gonova_tts_amd.config import vocoder_flops_per_sample

    B, T = args.batch, args.frames
    eng = HipEngine(local, vocoder_dtype=args.dtype, max_batch=B, max_frames=T)
    eng.load_weights(vocoder=make_vocoder_weights(seed=0))
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    mel = torch.randn((B, T, 80), generator=g).to(dev)
    lens = torch.full((B,), T, dtype=torch.int32, device=dev)
    wav = torch.empty((B, T * 256), dtype=torch.float32, device=dev)

    def step():
        eng.vocoder(mel, lens, out=wav)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    eng.profile(True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    eng.profile(False)
    gemm_ms, gemm_flops, n_launch = eng.profile_read()

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    samples_per_rank = B * T * 256 * args.steps
    total_samples = samples_per_rank * world
    value = total_samples / elapsed
    ms_per_step = elapsed * 1000.0 / args.steps
    per_gpu = value / world

    # roofline of the implicit-GEMM conv family (dominant kernel): algorithmic FLOPs per launch /
    # average launch duration, both from the timed region.
    per_launch_flops = gemm_flops / max(n_launch, 1)
    avg_launch_ms = gemm_ms / max(n_launch, 1)
    achieved = per_launch_flops / (avg_launch_ms * 1e-3) / 1e12 if n_launch else 0.0
    peak = MFMA_PEAK_TFLOPS[args.dtype]
    roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 5), "traffic": None,
            "kernel": "conv_gemm_kernel (implicit-GEMM conv, all vocoder launches)",
            "avg_launch_us": round(avg_launch_ms * 1e3, 2), "launches_per_step": n_launch // args.steps,
            "gemm_share_of_step": round(gemm_ms / (elapsed * 1e3), 4)}

    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (mel ~ N(0,1), seeded fan-in weights; no checkpoint offline)",
        "config": {"workload": "C2 vocoder-only HiFi-GAN V1, batch-32 x 862 frames (10.0 s) per GPU",
                   "global_batch": B * world, "frames": T, "samples_per_utt": T * 256,
                   "parallelism": f"utterance-sharded dp{world} (no data-path collective)"},
        "per_gpu_samples_per_s": round(per_gpu, 1),
        "x_realtime_per_gpu": round(per_gpu / SR, 2),
        "rtf": round(SR / per_gpu, 6),
        "algorithmic_tflops": round(value * vocoder_flops_per_sample() / 1e12 / world, 2),
        "roofline": roof,
    }
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_frames)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
