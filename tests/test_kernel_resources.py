"""No kernel of the product library uses scratch memory (no VGPR spills, no private arrays):
read from the gfx950 code objects' metadata inside libtts_hip.so (tools/kernel_resources.py;
no GPU).  Scratch traffic on a hot kernel is per-lane HBM/L2 round trips inside its loop; the
round-4 findings were the 64-channel conv_xres tile (its fused post-LN tail's double buffer
indexed by a loop counter, 144 B/lane), the bf16 streaming upsampler (8 B/lane at 12 waves) and
the HiFi-GAN V3 C = 64 k = 5 pair (8-12 B/lane at three blocks per CU)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.fixture(scope="module")
def kernels():
    from gonova_tts_amd import engine
    if not os.path.exists(engine.LIB_PATH):
        from gonova_tts_amd.build import build
        build()
    from kernel_resources import kernels as read
    ks = read(engine.LIB_PATH)
    assert ks, "no gfx950 kernel metadata found in the library"
    return ks


def test_no_kernel_uses_scratch(kernels):
    bad = [(k["name"], k["scratch"], k["vgpr_spill"]) for k in kernels if k["scratch"] or k["vgpr_spill"]]
    assert not bad, f"kernels with scratch / VGPR spills: {bad}"


def test_hot_kernels_present(kernels):
    """the metadata covers the kernels the C2 / C3 / C5 paths launch"""
    names = " ".join(k["name"] for k in kernels)
    for k in ("mrf_pair_kernel", "mrf_chain_kernel", "upsample_stream_kernel", "conv_xres_kernel",
              "rel_attn_kernel", "conv_splitp_kernel"):
        assert k in names, k
