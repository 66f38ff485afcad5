"""Checkpoint loading: weight-norm folding for HiFi-GAN checkpoints
saved with weight norm on, in both torch naming schemes, and the no-pickle loaders."""
import numpy as np
import pytest
import torch

from gonova_tts_amd.model import fold_weight_norm, load_state_dict


def _wn_modules():
    torch.manual_seed(0)
    return {"conv_pre": torch.nn.Conv1d(80, 16, 7, padding=3),
            "upsampler.0": torch.nn.ConvTranspose1d(16, 8, 16, stride=8, padding=4)}


@pytest.mark.parametrize("api", ["weight_g", "parametrizations"])
def test_fold_weight_norm_matches_torch(api):
    mods = _wn_modules()
    sd, ref = {}, {}
    for name, m in mods.items():
        if api == "weight_g":
            m = torch.nn.utils.weight_norm(m)
            m.weight_g.data.uniform_(0.5, 2.0)   # g != ||v|| so folding is not a no-op
            m(torch.zeros(1, m.in_channels, 32))  # recompute .weight from g, v
        else:
            m = torch.nn.utils.parametrizations.weight_norm(m)
            m.parametrizations.weight.original0.data.uniform_(0.5, 2.0)
        ref[name + ".weight"] = m.weight.detach().numpy()
        for k, v in m.state_dict().items():
            sd[f"{name}.{k}"] = v.detach().numpy()
    folded = fold_weight_norm(sd)
    for k, w in ref.items():
        np.testing.assert_allclose(folded[k], w, rtol=1e-6, atol=1e-7)
    assert not any(k.endswith(("weight_g", "weight_v", "original0", "original1")) for k in folded)
    assert all(k in folded for k in ("conv_pre.bias", "upsampler.0.bias"))


def test_load_state_dict_folds_and_refuses_pickles(tmp_path):
    from safetensors.numpy import save_file
    v = np.random.default_rng(0).standard_normal((4, 3, 5)).astype(np.float32)
    g = np.full((4, 1, 1), 2.0, np.float32)
    save_file({"c.weight_g": g, "c.weight_v": v, "c.bias": np.zeros(4, np.float32)}, str(tmp_path / "m.safetensors"))
    sd = load_state_dict(str(tmp_path / "m.safetensors"))
    np.testing.assert_allclose(np.sqrt((sd["c.weight"] ** 2).sum(axis=(1, 2))), 2.0, rtol=1e-6)
    np.savez(tmp_path / "m.npz", **{"c.weight": v})
    assert np.array_equal(load_state_dict(str(tmp_path / "m.npz"))["c.weight"], v)
    with pytest.raises(ValueError):
        load_state_dict(str(tmp_path / "m.pt"))
