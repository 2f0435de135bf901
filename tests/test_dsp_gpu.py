"""HIP DSP kernels of the FM-radio pipeline (csrc/kernels/dsp.hip) against scipy.signal in float64: complex FIR with
zero initial state, the FM discriminator and the polyphase resampler, incl. long filters and burst sizes that are not
multiples of the kernels' blocks; plus the whole signal chain on the GPU vs on the CPU."""
import numpy as np
import pytest
import torch

from generativeaiexamples_amd.community.fm_asr import dsp
from generativeaiexamples_amd.community.fm_asr.pipeline import SdrParams, SignalChain

signal = pytest.importorskip("scipy.signal")
pytestmark = pytest.mark.gpu


def _burst(n, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 1e6
    x = np.exp(1j * 2 * np.pi * 75e3 * np.cumsum(np.sin(2 * np.pi * 900 * t)) / 1e6)
    return (x + 0.05 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)


@pytest.mark.parametrize("n,ntaps", [(62500, 101), (1000, 7), (5001, 4096), (3, 101)])
def test_fir_complex_matches_lfilter(n, ntaps):
    x = _burst(n, n)
    taps = dsp.firwin(ntaps, 100e3, fs=1e6) if ntaps > 7 else np.linspace(0.1, 0.7, ntaps)
    y = dsp.lowpass(taps, torch.from_numpy(x).cuda()).cpu().numpy()
    np.testing.assert_allclose(y, signal.lfilter(taps, [1.0], x.astype(np.complex128)), rtol=1e-4, atol=2e-5)


def test_fm_demod_and_resample_match_scipy():
    x = _burst(62500, 1)
    d = dsp.fm_demod(torch.from_numpy(x).cuda())
    dref = np.diff(np.unwrap(np.angle(x.astype(np.complex128))))
    np.testing.assert_allclose(d.cpu().numpy(), dref, atol=5e-5)
    dd = d.cpu().numpy().astype(np.float64)
    for up, down in ((2, 125), (1, 62), (3, 2), (160, 147)):
        r = dsp.resample_poly(d, up, down, gain=10.0).cpu().numpy()
        rref = 10.0 * signal.resample_poly(dd, up, down, window="hamming")
        assert r.shape == rref.shape, (up, down)
        np.testing.assert_allclose(r, rref, rtol=1e-4, atol=2e-4)


def test_signal_chain_gpu_matches_cpu():
    x = torch.from_numpy(_burst(62500, 2))
    g = SignalChain(SdrParams(), device="cuda")(x.cuda()).cpu()
    c = SignalChain(SdrParams(), device="cpu")(x)
    assert g.shape == c.shape
    np.testing.assert_allclose(g.numpy(), c.numpy(), rtol=1e-3, atol=1e-3)


def test_dfp_autoencoder_trains_on_gpu():
    """The community DFP autoencoder trains and scores on the GPU (PyTorch-ROCm) like on the CPU."""
    import pandas as pd

    from generativeaiexamples_amd.community.dfp import AEConfig, TabularAutoEncoder

    rng = np.random.default_rng(0)
    df = pd.DataFrame({"hour": rng.normal(10, 1, 1024), "app": rng.choice(["a", "b", "c"], 1024),
                       "vpn": rng.random(1024) < 0.1})
    ae = TabularAutoEncoder(AEConfig(encoder_layers=[64], decoder_layers=[64], optimizer="adam", learning_rate=3e-3),
                            device="cuda")
    hist = ae.fit(df, epochs=5)
    assert next(ae.net.parameters()).is_cuda and hist[-1] < hist[0]
    odd = pd.DataFrame({"hour": [2.0, 23.0], "app": ["zzz", "zzz"], "vpn": [True, True]})
    assert ae.get_results(odd)["mean_abs_z"].min() > ae.get_results(df.head(200))["mean_abs_z"].median()


def test_dfp_graphed_sgd_matches_eager():
    """The graph-replayed SGD steps (full 512-row batches) do the same updates as the eager torch.optim.SGD loop: with
    swap noise off both see the same batches, so the per-epoch losses agree; with noise on the loss still falls."""
    import pandas as pd

    from generativeaiexamples_amd.community.dfp import AEConfig, TabularAutoEncoder

    rng = np.random.default_rng(1)
    n = 4 * 512 + 100  # four graph replays' worth plus an eager tail batch
    df = pd.DataFrame({"x": rng.normal(0, 1, n), "y": rng.normal(5, 2, n), "app": rng.choice(list("abcdef"), n),
                       "ok": rng.random(n) < 0.8})
    cfg = dict(encoder_layers=[64], decoder_layers=[64], learning_rate=0.05, swap_probability=0.0)
    graphed = TabularAutoEncoder(AEConfig(**cfg), device="cuda")
    h_graph = graphed.fit(df, epochs=3)
    eager = TabularAutoEncoder(AEConfig(**cfg), device="cuda")
    eager._fit_graphed = eager._fit_eager  # same data, seeds and init: the eager SGD loop
    h_eager = eager.fit(df, epochs=3)
    np.testing.assert_allclose(h_graph, h_eager, rtol=2e-3)
    for a, b in zip(graphed.net.parameters(), eager.net.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-2, atol=1e-4)
    noisy = TabularAutoEncoder(AEConfig(**{**cfg, "swap_probability": 0.2}), device="cuda")
    h = noisy.fit(df, epochs=4)
    assert h[-1] < h[0]
