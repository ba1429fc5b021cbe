"""GPU parity of windows above 16384 samples (large_fft.hip: four-step
transform; SURVEY.md sec. 8f rank 4, the legacy InpFFTWindow menu up to
262144, L/WaveSpecZZ_1.0.4-new.mq5:657).

Bar as everywhere: per window max_k |P - P_ref| / max_k P_ref <= 1e-10 (fp64)
against the CPU restatement (whose radix-2 twiddle recurrence is the least
exact party at these sizes), <= 1e-5 (fp32); numpy.fft as an independent
exact reference for the fp64 transform itself.
"""
import numpy as np
import pytest

import oracle
from wavespec_amd import bridge, synth

pytestmark = pytest.mark.gpu

TOL = {"f64": 1e-10, "f32": 1e-5}
KALMAN = oracle.KALMAN_DEFAULTS


def gpu(series, n, hop, detrend="none", window="hann", period=0, prec="f64", output="power"):
    return bridge.spectrum_batch(series, n, hop, detrend, window, period, prec, output)


def ref(series, n, hop, detrend="none", window="hann", period=0, output="power"):
    return oracle.batch_spectrum(series, n, hop, detrend, window, period, kalman=KALMAN, output=output)


def np_power(series, n, hop, window="hann"):
    nw = 1 + (series.size - n) // hop
    i = np.arange(n)
    win = {"none": np.ones(n), "hann": 0.5 * (1 - np.cos(2 * np.pi * i / (n - 1)))}[window]
    x = np.stack([series[w * hop:w * hop + n] for w in range(nw)]) * win
    return np.abs(np.fft.fft(x, axis=1)[:, :n // 2]) ** 2


@pytest.mark.parametrize("n", [32768, 65536, 131072, 262144])
def test_large_sizes(gpu_session, n):
    s = synth.random_walk(3 * n + 17, seed=n % 1000)
    p = gpu(s, n, n)
    assert p.shape == (3, n // 2)
    assert oracle.rel_err(p, ref(s, n, n)) <= TOL["f64"]
    assert oracle.rel_err(p, np_power(s, n, n)) <= 1e-12


@pytest.mark.parametrize("detrend,period", [("none", 0), ("mean", 0), ("iir", 1024), ("iir", 37), ("kalman", 0)])
@pytest.mark.parametrize("window", ["none", "hann", "hamming", "blackman", "bartlett"])
def test_large_detrend_window_matrix(gpu_session, detrend, period, window):
    n = 65536
    s = synth.random_walk(2 * n + 5, seed=7)
    p = gpu(s, n, n, detrend, window, period)
    assert oracle.rel_err(p, ref(s, n, n, detrend, window, period)) <= TOL["f64"], (detrend, window)


@pytest.mark.parametrize("n", [32768, 262144])
@pytest.mark.parametrize("detrend,period", [("none", 0), ("mean", 0), ("iir", 1024), ("kalman", 0)])
def test_large_f32(gpu_session, n, detrend, period):
    s = synth.random_walk(2 * n, seed=11)
    p = gpu(s, n, n, detrend, "hann", period, prec="f32")
    s32 = s.astype(np.float32).astype(np.float64)
    assert oracle.rel_err(p, ref(s32, n, n, detrend, "hann", period)) <= TOL["f32"]


@pytest.mark.parametrize("n", [32768, 131072])
def test_large_packed(gpu_session, n):
    s = synth.random_walk(2 * n, seed=3)
    p = gpu(s, n, n, "none", "hann", output="packed")
    r = ref(s, n, n, "none", "hann", output="packed")
    assert p.shape == r.shape == (2, n)
    assert np.max(np.abs(p - r)) <= 1e-9 * np.max(np.abs(r))


@pytest.mark.parametrize("n,hop", [(32768, 1), (32768, 777), (65536, 40001), (131072, 131073)])
def test_large_hops(gpu_session, n, hop):
    """Overlapping windows, odd hops (unaligned pair loads), gaps."""
    s = synth.random_walk(4 * hop + n, seed=hop % 97)
    p = gpu(s, n, hop, "mean", "hann")
    assert p.shape[0] == 5
    assert oracle.rel_err(p, ref(s, n, hop, "mean", "hann")) <= TOL["f64"]


def test_large_chunks(gpu_session):
    """More windows than one chunk of column results (256 at N = 32768 fp64): chunk seams."""
    n, w = 32768, 300
    s = synth.random_walk(w * 2048 + n - 2048, seed=5)
    p = gpu(s, n, 2048, "iir", "hann", 1024)
    assert p.shape == (w, n // 2)
    assert oracle.rel_err(p, ref(s, n, 2048, "iir", "hann", 1024)) <= TOL["f64"]


@pytest.mark.parametrize("n,chunk,variant", [(262144, 5, 1), (131072, 1, 1), (32768, 100, 1),
                                             (32768, 1, 2), (32768, 2, 2), (131072, 1, 2)])
def test_large_set_chunk(gpu_session, n, chunk, variant):
    """wsp_plan_set_chunk: the two-pass path over other chunk lengths (ragged last chunk, one window per chunk)
    gives the same records as the library's chunking (the same kernels on other chunk boundaries).  Variant 2
    (the pipelined two-pass form, two Y buffers of chunk / 4 windows) at one and two windows per chunk: a
    one-window workspace cannot hold its second buffer, so the plan runs the plain chunk loop."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    nwin = 13 if n > 65536 else 211
    s = synth.random_walk(nwin * n, seed=n // 4096 + chunk)
    d_s = torch.from_numpy(s).to(dev)
    outs = []
    for c in (0, chunk):
        plan = bridge.Plan(0, n, n, nwin, "mean", "hann")
        plan.set_variant(variant if c else 1)  # the two-pass path (the reference run: variant 1, default chunk)
        plan.set_chunk(c)
        o = torch.empty(nwin * plan.record, dtype=torch.float64, device=dev)
        plan.execute(d_s.data_ptr(), o.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append(o.cpu().numpy().reshape(nwin, plan.record))
        plan.close()
    assert np.array_equal(outs[0], outs[1])
    assert oracle.rel_err(outs[1][:2], ref(s[:2 * n], n, n, "mean", "hann", 0)) <= TOL["f64"]


def test_large_fft_real_forward(gpu_session):
    """gpu_fft_real_forward at the legacy default InpFFTWindow = 65536."""
    n = 65536
    x = synth.random_walk(n, seed=1)
    packed = bridge.fft_real_forward(x)
    re, im = oracle.fft_manual(x)
    scale = np.max(np.abs(re[:n // 2]))
    assert np.max(np.abs(packed[0::2] - re[:n // 2])) <= 1e-10 * scale
    assert np.max(np.abs(packed[1::2] - im[:n // 2])) <= 1e-10 * scale


def test_large_rejects_topk_and_inverse(gpu_session):
    n = 32768
    s = synth.random_walk(2 * n, seed=2)
    with pytest.raises(bridge.BridgeError) as e:
        bridge.spectrum_topk_batch(s, n, n, "none", "hann", top_k=8, min_period=18.0, max_period=200.0)
    assert e.value.status == -1
    with pytest.raises(bridge.BridgeError) as e:
        bridge.fft_real_inverse(np.zeros(n))
    assert e.value.status == -1


def test_large_device_plan(gpu_session):
    """wsp_plan_* at N = 65536 over 64 windows (chunked column results in the plan workspace)."""
    import torch
    n, w = 65536, 64
    s = synth.random_walk(w * n, seed=9)
    plan = bridge.Plan(0, n, n, w, "kalman", "hann")
    try:
        d_s = torch.from_numpy(s).cuda()
        d_o = torch.empty(w * (n // 2), dtype=torch.float64, device="cuda")
        plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        p = d_o.cpu().numpy().reshape(w, n // 2)
    finally:
        plan.close()
    assert oracle.rel_err(p[:8], ref(s[:8 * n], n, n, "kalman", "hann")) <= TOL["f64"]
    assert oracle.rel_err(p[-4:], ref(s[-4 * n:], n, n, "kalman", "hann")) <= TOL["f64"]


@pytest.mark.parametrize("n,variant,detrend,window,output", [
    (65536, 0, "none", "hann", "power"), (65536, 0, "mean", "bartlett", "packed"), (65536, 0, "iir", "hamming", "power"),
    (65536, 2, "none", "hann", "power"), (65536, 3, "none", "hann", "power"), (65536, 3, "mean", "blackman", "packed"),
    (65536, 4, "none", "hann", "power"), (65536, 5, "mean", "hann", "power"), (131072, 3, "none", "bartlett", "power"),
    (131072, 2, "iir", "hann", "power"), (262144, 6, "none", "hann", "power"), (262144, 6, "mean", "blackman", "packed"),
    (262144, 7, "none", "hann", "power"), (32768, 7, "iir", "bartlett", "packed"),
    (32768, 2, "mean", "hamming", "power"), (65536, 8, "none", "hann", "power"), (65536, 8, "mean", "blackman", "packed"),
    (131072, 8, "iir", "hamming", "power")])
def test_large_variants_identical(gpu_session, n, variant, detrend, window, output):
    """The large-N kernel forms (wsp_plan_set_variant) against the two-pass form (variant 1): 0 = the library's
    choice (the fused kernel for fp64 N = 65536), 2 = two-pass over quarter chunks pipelined on two internal
    streams, 3 = the fused one-workgroup-per-window kernel at 512 threads, 4 = the same at 256 threads with
    register prefetch, 5 = the fused kernel with plain output stores, 6 = N = 262144's column pass at 16 columns
    per workgroup (the default takes 8), 7 = the two-pass row kernel in plain block order (the default maps blocks
    XCD-aware), 8 = two passes with 8-column column workgroups at M2 = 256 (N = 65536 / 131072).  They run the
    same arithmetic: identical records (variants 2, 6, 7 and 8) or
    within 1e-13 (the fused kernel: the same operations, contracted differently by the
    compiler; its window angles by rotation across column blocks), and the oracle's bar."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    nwin = 37
    s = synth.random_walk(nwin * n, seed=n // 1024 + variant)
    d_s = torch.from_numpy(s).to(dev)
    period = 1024 if detrend == "iir" else 0
    outs = []
    for v in (1, variant):
        plan = bridge.Plan(0, n, n, nwin, detrend, window, period, "f64", output)
        plan.set_variant(v)
        o = torch.empty(nwin * plan.record, dtype=torch.float64, device=dev)
        plan.execute(d_s.data_ptr(), o.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append(o.cpu().numpy().reshape(nwin, plan.record))
        plan.close()
    if variant in (2, 6, 7, 8):  # the same per-column arithmetic over other chunk boundaries / workgroup shapes: identical
        assert np.array_equal(outs[0], outs[1])
    else:
        den = np.abs(outs[0]).max(axis=1, keepdims=True)
        assert np.max(np.abs(outs[1] - outs[0]) / den) <= 1e-13
    if output == "power":
        assert oracle.rel_err(outs[1][:4], ref(s[:4 * n], n, n, detrend, window, period)) <= TOL["f64"]


def test_large_fused_more_windows_than_slots(gpu_session):
    """The default fused kernel (fp64, N = 65536) walks windows g, g + grid, ... over its slots: a batch of
    more windows than workgroups (600 > 256 CUs) with a ragged tail, against the oracle on sampled windows."""
    torch = pytest.importorskip("torch")
    n, nwin = 65536, 600
    s = synth.random_walk(nwin * 4096 + n, seed=21)
    plan = bridge.Plan(0, n, 4096, nwin, "none", "hann")
    try:
        d_s = torch.from_numpy(s).cuda()
        d_o = torch.empty(nwin * (n // 2), dtype=torch.float64, device="cuda")
        plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        p = d_o.cpu().numpy().reshape(nwin, n // 2)
    finally:
        plan.close()
    for w in (0, 255, 256, 511, 599):
        r = ref(s[w * 4096:w * 4096 + n], n, n)
        assert oracle.rel_err(p[w:w + 1], r) <= TOL["f64"], w
