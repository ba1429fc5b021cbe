"""GPU parity: libmtbridge.so (HIP, gfx950) against the CPU restatement.

Bar: per window
max_k |P - P_ref| / max_k P_ref <= 1e-10 for fp64 and <= 1e-5 for fp32.
All calls go through the C ABI.
"""
import ctypes as C
import subprocess

import numpy as np
import pytest

import oracle
from conftest import ROOT
from wavespec_amd import bridge, indicator, synth

pytestmark = pytest.mark.gpu

TOL = {"f64": 1e-10, "f32": 1e-5}
KALMAN = oracle.KALMAN_DEFAULTS


def gpu(series, n, hop, detrend="none", window="hann", period=0, prec="f64", output="power"):
    return bridge.spectrum_batch(series, n, hop, detrend, window, period, prec, output)


def ref(series, n, hop, detrend="none", window="hann", period=0, output="power"):
    return oracle.batch_spectrum(series, n, hop, detrend, window, period, kalman=KALMAN, output=output)


@pytest.mark.parametrize("n", [32, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384])
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_sizes_hann(gpu_session, n, prec):
    s = synth.random_walk(37 * n + 11, seed=n)
    p = gpu(s, n, n, prec=prec)
    r = ref(s.astype(np.float32).astype(np.float64) if prec == "f32" else s, n, n)
    assert p.shape == r.shape == (37, n // 2)
    assert oracle.rel_err(p, r) <= TOL[prec]
    if prec == "f64":  # the cycle bins to the same bar (rel_err is normalised by P_0 here)
        assert oracle.inband_err(p, r, *oracle.band(n)) <= TOL[prec]


@pytest.mark.parametrize("n", [64, 1024, 4096, 16384])
@pytest.mark.parametrize("detrend,period", [("none", 0), ("mean", 0), ("iir", 1024), ("iir", 37), ("kalman", 0)])
@pytest.mark.parametrize("window", ["none", "hann", "hamming", "blackman", "bartlett"])
def test_detrend_window_matrix(gpu_session, n, detrend, period, window):
    s = synth.random_walk(9 * n, seed=3 * n + period)
    p = gpu(s, n, n, detrend, window, period)
    r = ref(s, n, n, detrend, window, period)
    assert oracle.rel_err(p, r) <= TOL["f64"], (detrend, window)
    assert oracle.inband_err(p, r, *oracle.band(n)) <= TOL["f64"], (detrend, window)


@pytest.mark.parametrize("detrend,period", [("none", 0), ("mean", 0), ("iir", 1024), ("kalman", 0)])
def test_f32_detrends(gpu_session, detrend, period):
    """fp32 path: the series is stored as float (C3), so the oracle gets the
    same float-rounded prices.  (Against the unrounded fp64 series the Kalman
    residual -- ~1e-5 on prices ~1.1 -- carries the input rounding itself:
    ~4e-5, a property of fp32 storage, not of the FFT.)"""
    n = 4096
    s = synth.random_walk(6 * n, seed=11)
    p = gpu(s, n, n, detrend, "hann", period, prec="f32")
    s32 = s.astype(np.float32).astype(np.float64)
    assert oracle.rel_err(p, ref(s32, n, n, detrend, "hann", period)) <= TOL["f32"]


@pytest.mark.parametrize("n,hop", [(2048, 1), (1024, 3), (256, 1), (4096, 4097), (512, 700), (64, 1), (16384, 1),
                                   (8192, 333)])
def test_overlap_and_unaligned_hops(gpu_session, n, hop):
    """hop=1 (C4 shape, odd offsets -> unaligned loads), hop > N (gaps)."""
    s = synth.random_walk((150 - 1) * hop + n, seed=13)
    p = gpu(s, n, hop)
    r = ref(s, n, hop)
    assert p.shape[0] == 150
    assert oracle.rel_err(p, r) <= TOL["f64"]


@pytest.mark.parametrize("nwin", [1, 2, 3, 127, 129, 1000])
def test_ragged_window_counts(gpu_session, nwin):
    """Window counts that do not fill the last workgroup (2048/M windows per group)."""
    n = 64
    s = synth.random_walk(nwin * n, seed=nwin)
    assert oracle.rel_err(gpu(s, n, n, "mean"), ref(s, n, n, "mean")) <= TOL["f64"]


@pytest.mark.parametrize("n", [32, 1024, 4096, 16384])
def test_packed_output(gpu_session, n):
    s = synth.random_walk(5 * n, seed=5)
    p = gpu(s, n, n, "none", "hann", output="packed")
    r = ref(s, n, n, "none", "hann", output="packed")
    scale = np.max(np.abs(r), axis=1, keepdims=True)
    assert np.max(np.abs(p - r) / scale) < 1e-12
    assert np.all(p[:, 1] == 0.0)  # Im X_0


def test_fft_real_forward_matches_cpu_fallback(gpu_session):
    """gpu_fft_real_forward vs FourierTransformManual (the CPU fallback the
    callers swap it for: L/WaveSpecZZ_1.0.4-new.mq5:3174-3208)."""
    x = synth.sine_noise_window(1024)
    out = bridge.fft_real_forward(x)
    re, im = oracle.fft_manual(x)
    assert np.max(np.abs(out[0::2] - re[:512])) / np.max(np.abs(re)) < 1e-13
    assert np.max(np.abs(out[1::2] - im[:512])) / np.max(np.abs(re)) < 1e-13


def test_fft_real_forward_batch(gpu_session):
    w = synth.random_walk(8 * 512, seed=1).reshape(8, 512)
    out = bridge.fft_real_forward_batch(w)
    for i in range(8):
        assert np.allclose(out[i], bridge.fft_real_forward(w[i]), rtol=0, atol=1e-12)


def test_out_cap_truncates_records(gpu_session):
    s = synth.random_walk(10 * 256, seed=2)
    out = np.full((10, 128), -1.0)
    got = C.c_int32(0)
    st = bridge.lib().gpu_spectrum_batch(bridge._dptr(s), s.size, 256, 256, 0, 1, 0, 0, 0, bridge._dptr(out),
                                         4 * 128 + 5, C.byref(got))
    assert st == bridge.OK and got.value == 4
    assert np.all(out[4:] == -1.0)
    assert oracle.rel_err(out[:4], ref(s, 256, 256)[:4]) <= 1e-10


def test_async_job_api(gpu_session):
    s = synth.random_walk(20000, seed=21)
    p = indicator.batch_spectra(s, 1024, 1, "iir", "hann", 1024)
    assert p.shape == (20000 - 1024 + 1, 512)
    idx = np.r_[0:50, 9000:9050, p.shape[0] - 50:p.shape[0]]
    r = np.stack([oracle.window_spectrum(s[i:i + 1024], "iir", "hann", 1024) for i in idx])
    assert oracle.rel_err(p[idx], r) <= 1e-10


def test_async_submit_copies_input(gpu_session):
    s = synth.random_walk(8192, seed=4)
    keep = s.copy()
    jid = bridge.submit_spectrum_batch(s, 1024, 1024)
    s[:] = 0.0  # caller reuses its buffer right after submit (1.1.0:1316)
    out = np.empty((8, 512))
    for _ in range(20000):
        st, ready, n = bridge.try_get_spectrum_batch(jid, out)
        if ready:
            break
    assert st == bridge.OK and ready == 1 and n == 8
    assert bridge.free_job(jid) == bridge.OK
    assert bridge.free_job(jid) == bridge.BAD_ARGS
    assert oracle.rel_err(out, ref(keep, 1024, 1024)) <= 1e-10


def test_feed_pipeline_on_calculate(gpu_session, tmp_path):
    """FeedCache file -> FeedBuilder -> FftProcessor per bar, as 1.1.0 does."""
    n, bars = 512, 40
    hist = synth.random_walk(n + bars - 1 + 100, seed=8)
    close = hist[::-1].copy()  # newest first
    cache = indicator.FeedCache()
    ok, delta, _ = indicator.ensure_feed_cache(cache, "EURUSD", "M1", n + bars, True, "WaveSpecZZ",
                                               lambda start, cnt: close[start:start + cnt], str(tmp_path))
    assert ok and delta == n + bars
    spectra = indicator.on_calculate(cache, n, bars)
    for b in (0, bars // 2, bars - 1):
        shift = bars - 1 - b
        win = close[shift:shift + n][::-1]
        assert oracle.rel_err(spectra[b], oracle.window_spectrum(win, "none", "none")) <= 1e-10


@pytest.mark.parametrize("mode", ["live", "batch"])
def test_cpp_harness(gpu_session, tmp_path, mode):
    """The C++ MT5 stand-in dlopen()s the library and runs the reference call sequences."""
    n, bars = 1024, 64
    hist = synth.random_walk(n + bars - 1, seed=31)
    feed = tmp_path / "feed.bin"
    indicator.save_feed_cache(str(feed), hist[::-1].copy())
    out = tmp_path / "out.bin"
    r = subprocess.run([str(ROOT / "fft-wavespec_amd" / "bin" / "oncalculate_harness"), str(bridge.LIB_PATH), mode,
                        str(feed), str(n), str(bars), str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    spectra = np.fromfile(out, dtype=np.float64).reshape(bars, n // 2)
    want = ref(hist, n, 1, "none", "none")
    assert oracle.rel_err(spectra, want) <= 1e-10


def test_plan_device_resident(gpu_session):
    torch = pytest.importorskip("torch")
    n, w = 4096, 512
    dev = torch.device("cuda", 0)
    s = synth.random_walk(n * w, seed=11)
    d_s = torch.from_numpy(s).to(dev)
    d_o = torch.empty(w * n // 2, dtype=torch.float64, device=dev)
    plan = bridge.Plan(0, n, n, w, "none", "hann")
    assert plan.algorithmic_bytes == (n * w + w * n // 2) * 8
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    p = d_o.cpu().numpy().reshape(w, n // 2)
    idx = np.r_[0:8, w - 8:w]
    assert oracle.rel_err(p[idx], ref(s[: (idx[-1] + 1) * n], n, n)[idx]) <= 1e-10
    plan.close()


def test_full_size_properties(gpu_session):
    """North-star size (65536 x 4096 fp64, 3 GB moved) with the mean detrend and the Blackman window
    (the kWinCos2 instantiation; the benchmarked Hann one: test_gpu_fullgrid.py): size-independent
    properties over ALL windows + oracle parity on windows of both grid-stride iterations."""
    torch = pytest.importorskip("torch")
    n, w = 4096, 65536
    dev = torch.device("cuda", 0)
    d_s = synth.random_walk_torch(n * w, 11, dev)
    d_o = torch.empty(w * n // 2, dtype=torch.float64, device=dev)
    plan = bridge.Plan(0, n, n, w, "mean", "blackman")
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    P = d_o.view(w, n // 2)
    X = d_s.view(w, n)
    i = torch.arange(n, device=dev, dtype=torch.float64)
    bl = 0.42 - 0.5 * torch.cos(2 * np.pi * i / (n - 1)) + 0.08 * torch.cos(4 * np.pi * i / (n - 1))
    Xs = X[::257]
    F = torch.fft.rfft((Xs - Xs.mean(dim=1, keepdim=True)) * bl, dim=1)[:, : n // 2]
    Pt = F.real ** 2 + F.imag ** 2
    err = ((P[::257] - Pt).abs().amax(dim=1) / Pt.abs().amax(dim=1)).max().item()
    assert err < 1e-12
    assert torch.isfinite(P).all().item() and (P >= 0).all().item()
    sel = [0, 12345, 32767, 32768, 50000, w - 1]  # 32768 workgroups: w >= 32768 is the second iteration
    host = d_s.view(w, n)[sel].cpu().numpy()
    got = P[sel].cpu().numpy()
    want = np.stack([oracle.window_spectrum(x, "mean", "blackman") for x in host])
    assert oracle.rel_err(got, want) <= 1e-10
    assert oracle.inband_err(got, want, *oracle.band(n)) <= 1e-10
    plan.close()


def test_multi_device_session_shards(gpu_session):
    """gpu_init(-1): windows sharded over every visible GPU (1 on the test box)."""
    bridge.shutdown()
    bridge.init(-1, 16)
    try:
        s = synth.random_walk(300 * 512, seed=17)
        assert oracle.rel_err(gpu(s, 512, 512), ref(s, 512, 512)) <= 1e-10
    finally:
        bridge.shutdown()
        bridge.init(0, 16)


@pytest.mark.parametrize("path", sorted((ROOT / "tests" / "golden").glob("*.npz")), ids=lambda p: p.stem)
def test_golden_vectors_on_gpu(gpu_session, path):
    g = np.load(path, allow_pickle=False)
    p = gpu(g["series"], int(g["n"]), int(g["hop"]), str(g["detrend"]), str(g["window"]), int(g["trend_period"]))
    assert oracle.rel_err(p, g["power"]) <= 1e-10


def _topk_match(got, want, tol, full_max):
    """Bins identical except where two candidates' powers tie within tol (the order of a near-tie
    is decided by rounding); powers and Re/Im within tol -- normalised, like every parity check
    here, by the window's full-spectrum max power."""
    assert got.shape == want.shape
    for w in range(got.shape[0]):
        gb, wb = got[w, :, 0].astype(int), want[w, :, 0].astype(int)
        scale = max(full_max[w], 1e-300)
        for s in np.nonzero(gb != wb)[0]:
            assert abs(got[w, s, 1] - want[w, s, 1]) <= tol * scale, (w, s, gb, wb)
        assert np.max(np.abs(got[w, :, 1] - want[w, :, 1])) <= tol * scale
        amp = max(np.sqrt(scale), 1e-300)
        same = gb == wb
        assert np.max(np.abs(got[w, same, 2:] - want[w, same, 2:]), initial=0.0) <= tol * amp * 10


@pytest.mark.parametrize("n", [2048, 4096])
@pytest.mark.parametrize("detrend,window,hop_of", [("none", "hann", "n"), ("none", "blackman", "1"),
                                                   ("mean", "hamming", "37"), ("none", "none", "n+5"),
                                                   ("mean", "bartlett", "n/4")])
def test_phase_split_form(gpu_session, n, detrend, window, hop_of):
    """Round 5: the split-exchange phase record (wsp_plan_set_variant 2 at N = 2048 / 4096 without IIR: Re and Im of X
    staged through the 17 KiB split slot one after the other, the three rows written one after another, atan2 with
    its coefficients in SGPRs -- 3 waves per SIMD; an ablation, slower than the default) against the AoS form (the
    default) and the oracle, over every window: power rows to 1e-13 of each other (the forms evaluate the cosine
    windows differently) and both to the oracle's 1e-10; phases and delays by the unwrap / delay bars of
    test_phase_output."""
    torch = pytest.importorskip("torch")
    hop = {"1": 1, "37": 37, "n/4": n // 4, "n": n, "n+5": n + 5}[hop_of]
    nwin = 90
    s = synth.random_walk((nwin - 1) * hop + n, seed=n + hop)
    dev = torch.device("cuda", 0)
    d_s = torch.from_numpy(s).to(dev)
    outs = []
    for v in (2, 0):
        plan = bridge.Plan(0, n, hop, nwin, detrend, window, output="phase")
        plan.set_variant(v)
        d_o = torch.full((nwin * 3 * (n // 2),), float("nan"), dtype=torch.float64, device=dev)
        plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append(d_o.view(nwin, 3, n // 2).cpu().numpy())
        plan.close()
    split, aos = outs
    assert np.isfinite(split).all()
    scale = aos[:, 0].max(axis=1, keepdims=True)
    assert np.all(np.abs(split[:, 0] - aos[:, 0]) <= 1e-13 * scale)
    want = oracle.batch_phase(s, n, hop, detrend, window)
    for got in outs:
        assert oracle.rel_err(got[:, 0], want[:, 0]) <= 1e-10
        for w in range(nwin):
            mag = np.sqrt(want[w, 0])
            m = _unwrap_match(got[w, 1], want[w, 1], mag)
            _delay_match(got[w, 2], want[w, 2], mag, m)


@pytest.mark.parametrize("n,hop,k,minp,maxp", [(4096, 4096, 8, 18, 200), (1024, 1, 8, 9, 200), (64, 7, 3, 4, 64),
                                               (256, 256, 16, 2, 10000), (512, 512, 8, 300, 400),
                                               (16384, 16384, 8, 18, 52), (8192, 100, 64, 2, 8192)])
@pytest.mark.parametrize("detrend", ["none", "iir"])
def test_topk_scan(gpu_session, n, hop, k, minp, maxp, detrend):
    """Fused top-k bin scan (gpuopt-nodetrend.mq5:536-554) against the oracle."""
    s = synth.random_walk((40 - 1) * hop + n, seed=n + k)
    got = bridge.spectrum_topk_batch(s, n, hop, detrend, "hann", 1024, "f64", k, minp, maxp)
    want = oracle.batch_topk(s, n, hop, detrend, "hann", 1024, None, k, minp, maxp)
    _topk_match(got, want, 1e-10, ref(s, n, hop, detrend, "hann", 1024).max(axis=1))


def test_topk_f32_and_plan(gpu_session):
    torch = pytest.importorskip("torch")
    n, w = 2048, 300
    s = synth.random_walk(n * w, seed=3)
    got = bridge.spectrum_topk_batch(s, n, n, "none", "hann", 0, "f32", 8, 18, 200)
    s32 = s.astype(np.float32).astype(np.float64)
    want = oracle.batch_topk(s32, n, n, "none", "hann", 0, None, 8, 18, 200)
    _topk_match(got, want, 1e-5, ref(s32, n, n).max(axis=1))
    plan = bridge.Plan(0, n, n, w, "none", "hann")
    plan.set_topk(8, 18, 200)
    d_s = torch.from_numpy(s).cuda()
    d_o = torch.empty(w * 32, dtype=torch.float64, device="cuda")
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    _topk_match(d_o.cpu().numpy().reshape(w, 8, 4), oracle.batch_topk(s, n, n, "none", "hann", 0, None, 8, 18, 200),
                1e-10, ref(s, n, n).max(axis=1))
    plan.close()


@pytest.mark.parametrize("window", ["hann", "blackman"])
def test_topk_f32_kalman_window_fold(gpu_session, window):
    """fp32 Kalman top-k records: the filter folds the window into its rows (kalman_folds_window) and the top-k launch
    runs unwindowed -- bins, powers and Re/Im of the winners as the oracle's windowed spectrum at the fp32 bar."""
    n, w = 2048, 200
    s = synth.random_walk(n * w, seed=29)
    s32 = s.astype(np.float32).astype(np.float64)
    got = bridge.spectrum_topk_batch(s32, n, n, "kalman", window, 0, "f32", 8, 18, 200)
    want = oracle.batch_topk(s32, n, n, "kalman", window, 0, None, 8, 18, 200)
    _topk_match(got, want, 1e-5, ref(s32, n, n, "kalman", window).max(axis=1))


# ---------------------------------------------------------------- inverse + phase
def _nyquist_free(x):
    n = x.shape[-1]
    alt = (-1.0) ** np.arange(n)
    return x - np.outer(x @ alt, alt).reshape(x.shape) / n


@pytest.mark.parametrize("n", [32, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384])
def test_inverse_batch_vs_oracle(gpu_session, n):
    """gpu_fft_real_inverse_batch (L/WaveSpecZZ_1.0.4-core.mq5:65,426) on random packed spectra,
    ragged window count; bar: max |x - x_ref| <= 1e-12 * max |x_ref| (fp64 round-off of two FFTs)."""
    rng = np.random.default_rng(n)
    w = 37
    spec = rng.standard_normal((w, n))
    got = bridge.fft_real_inverse_batch(spec)
    for i in range(w):
        want = oracle.fft_real_inverse(spec[i])
        assert np.max(np.abs(got[i] - want)) <= 1e-12 * np.max(np.abs(want)), i


@pytest.mark.parametrize("n", [32, 1024, 4096, 16384])
def test_inverse_round_trip_single(gpu_session, n):
    """gpu_fft_real_inverse(gpu_fft_real_forward(x)) == x (x without a Nyquist component), the
    round trip ApplySpectralStages makes (core.mq5:344 -> :426)."""
    x = _nyquist_free(synth.random_walk(n, n))
    back = bridge.fft_real_inverse(bridge.fft_real_forward(x))
    assert np.max(np.abs(back - x)) <= 1e-13 * np.max(np.abs(x))


@pytest.mark.parametrize("n", [1024, 2048, 4096, 8192])
def test_inverse_forms(gpu_session, n):
    """The inverse plan's kernel forms (wsp_plan_set_variant): 0 = the C2R pre-step in registers with the split
    exchange (default at N = 2048 .. 8192; each element's two reads paired in time, round 5), 1 = the pre-step
    through LDS (round-1 form), 2 = registers + the AoS exchange, 3 = the default with the loads in natural order
    (round 4; bit-identical to 0: only the load order differs), 4 = the default with plain stores (bit-identical): each against the oracle (1e-12 of the window's max)
    and within 1e-14 of each other, on a ragged batch (the last workgroup's window slots past the end)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(n + 1)
    w = 333
    spec = rng.standard_normal((w, n))
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(spec).to(dev)
    outs = []
    for v in (0, 1, 2, 3, 4):
        plan = bridge.Plan.inverse(0, n, w)
        plan.set_variant(v)
        d_o = torch.full((w * n,), float("nan"), dtype=torch.float64, device=dev)
        plan.execute(d_in.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append(d_o.view(w, n).cpu().numpy())
        plan.close()
    for i in range(0, w, 17):
        want = oracle.fft_real_inverse(spec[i])
        for o in outs:
            assert np.max(np.abs(o[i] - want)) <= 1e-12 * np.max(np.abs(want)), i
    scale = np.abs(outs[1]).max(axis=1, keepdims=True)
    assert np.all(np.abs(outs[0] - outs[1]) <= 1e-14 * scale)
    assert np.all(np.abs(outs[2] - outs[1]) <= 1e-14 * scale)
    if n >= 2048:
        assert np.array_equal(outs[3], outs[0])
        assert np.array_equal(outs[4], outs[0])


def test_inverse_plan_full_size(gpu_session):
    """Device-resident forward (packed) -> inverse plans over 65536 x 4096 fp64 (2 GiB each way):
    round trip returns x minus its Nyquist component for every window."""
    torch = pytest.importorskip("torch")
    n, w = 4096, 65536
    dev = torch.device("cuda", 0)
    d_x = synth.random_walk_torch(n * w, 5, dev)
    d_spec = torch.empty(w * n, dtype=torch.float64, device=dev)
    d_back = torch.empty(w * n, dtype=torch.float64, device=dev)
    fwd = bridge.Plan(0, n, n, w, "none", "none", output="packed")
    inv = bridge.Plan.inverse(0, n, w)
    assert inv.algorithmic_bytes == 2 * n * w * 8
    stream = torch.cuda.current_stream().cuda_stream
    fwd.execute(d_x.data_ptr(), d_spec.data_ptr(), stream)
    inv.execute(d_spec.data_ptr(), d_back.data_ptr(), stream)
    torch.cuda.synchronize()
    X, Y = d_x.view(w, n), d_back.view(w, n)
    alt = torch.ones(n, dtype=torch.float64, device=dev)
    alt[1::2] = -1.0
    want = X - (X @ alt)[:, None] * alt[None, :] / n
    err = ((Y - want).abs().amax(dim=1) / want.abs().amax(dim=1)).max().item()
    assert err <= 1e-13
    fwd.close()
    inv.close()


def _phase_tol(mag, rel=1e-10):
    """A phase computed from X_k carries |dX| / |X_k| of error: with |dX| ~ 1e-13 max |X| (the
    spectra's own fp64 parity), bar = rel * max|X| / |X_k| (1000x margin), never below rel."""
    return rel * np.maximum(mag.max() / np.maximum(mag, 1e-300), 1.0)


def _unwrap_match(got, want, mag):
    """Unwrapped phases agree within _phase_tol on well-conditioned bins (|X_k| >= 1e-9 max |X|);
    a 2 pi offset is allowed only after an ill-conditioned bin, whose phase is rounding noise and
    whose jump decision therefore is too (e.g. X_0 of a mean-removed window)."""
    ok = mag >= 1e-9 * mag.max()
    d = got - want
    m = np.round(d / (2 * np.pi))
    assert np.all((np.abs(d - 2 * np.pi * m) <= _phase_tol(mag))[ok])
    steps = np.nonzero(np.diff(m) != 0)[0] + 1
    for k in steps:
        assert not (ok[k] and ok[k - 1]), k
    return m


def _delay_match(got, want, mag, m):
    """Group delay = differences of neighbouring unwrapped phases: bar from the worse neighbour."""
    ok = mag >= 1e-9 * mag.max()
    tol = _phase_tol(mag)
    tn = tol.copy()
    tn[1:] = np.maximum(tn[1:], tol[:-1])
    tn[:-1] = np.maximum(tn[:-1], tol[1:])
    cond = ok.copy()
    cond[1:-1] &= ok[:-2] & ok[2:] & (m[:-2] == m[2:])
    assert np.all((np.abs(got - want) <= tn)[cond])


@pytest.mark.parametrize("n", [32, 256, 1024, 2048, 4096, 16384])
@pytest.mark.parametrize("detrend,period", [("none", 0), ("mean", 0), ("iir", 1024)])
def test_phase_output(gpu_session, n, detrend, period):
    """MTB_OUT_PHASE: [P | unwrapped phase | group delay] (1.0.4-new.mq5:1040-1120 at :3225-3227)."""
    hop = n // 2 + 3
    s = synth.random_walk(24 * hop + n, seed=n + 3)
    got = gpu(s, n, hop, detrend, "hann", period, output="phase")
    nwin = got.shape[0]
    got = got.reshape(nwin, 3, n // 2)
    want = oracle.batch_phase(s, n, hop, detrend, "hann", period)
    assert oracle.rel_err(got[:, 0], want[:, 0]) <= 1e-10
    for w in range(nwin):
        mag = np.sqrt(want[w, 0])
        m = _unwrap_match(got[w, 1], want[w, 1], mag)
        _delay_match(got[w, 2], want[w, 2], mag, m)


@pytest.mark.parametrize("n,hop,k,minp,maxp", [(4096, 4096, 8, 18, 200), (1024, 1, 8, 9, 200), (64, 7, 3, 4, 64),
                                               (16384, 4000, 8, 18, 52),
                                               # bins per thread of the phase scan (2/4/8/16 by kmax): CH = 8, 16, 8
                                               (4096, 4096, 8, 6, 200), (4096, 4096, 5, 3, 300), (2048, 1, 8, 5, 100)])
def test_topk_phase(gpu_session, n, hop, k, minp, maxp):
    """MTB_OUT_TOPK_PHASE: top-k records + unwrapped phase / group delay at each chosen bin (the
    values ComputeETA_RealFFT / CalculateScientificETASeconds read, 1.0.4-new.mq5:1165, :1239)."""
    s = synth.random_walk((30 - 1) * hop + n, seed=n + k + 1)
    got = bridge.spectrum_topk_phase_batch(s, n, hop, "iir", "hann", 1024, k, minp, maxp)
    want = oracle.batch_topk_phase(s, n, hop, "iir", "hann", 1024, None, k, minp, maxp)
    _topk_match(got[:, :, :4], want[:, :, :4], 1e-10, ref(s, n, hop, "iir", "hann", 1024).max(axis=1))
    full = oracle.batch_phase(s, n, hop, "iir", "hann", 1024)
    for w in range(got.shape[0]):
        mag = np.sqrt(full[w, 0])
        ok = mag >= 1e-9 * mag.max()
        same = (got[w, :, 0] == want[w, :, 0]) & (want[w, :, 0] >= 0)
        b = want[w, same, 0].astype(int)
        if ok[: max(b.max(initial=0), 1) + 2].all():  # no ill-conditioned bin up to the chosen ones
            assert np.max(np.abs(got[w, same, 4:] - want[w, same, 4:]), initial=0.0) <= 1e-8


@pytest.mark.parametrize("n,k,minp,maxp,window", [(4096, 8, 18, 200, "hann"), (2048, 8, 18, 200, "hann"),
                                                  (4096, 8, 6, 200, "hamming"), (4096, 5, 3, 300, "hann"),
                                                  (2048, 8, 4.1, 2000, "none"), (4096, 64, 18, 200, "blackman"),
                                                  (2048, 1, 9, 30, "hann"), (4096, 8, 100, 110, "hann")])
def test_topk_phase_split_form(gpu_session, n, k, minp, maxp, window):
    """MTB_OUT_TOPK_PHASE without detrend at N = 2048 / 4096 (ns_topk_phase's instantiation): the split-exchange
    form (one-wave scan, then one wave for the winners' phases: geometric unwrap decisions, atan2 only at each
    winner and its neighbours) against the AoS form (wsp_plan_set_variant 1: every thread's phase chunk) -- the
    same bins and powers to 1e-12 -- and both against the oracle (phases and delays to 1e-8).  Bands whose bins
    0 .. kmax + 1 take 2 / 4 / 8 / 16 bins per lane, and one beyond the split slot (periods 3-300: the AoS form)."""
    _topk_phase_forms(n, k, minp, maxp, window, n)


@pytest.mark.parametrize("n,window", [(4096, "hann"), (2048, "blackman")])
@pytest.mark.parametrize("hop_of", ["1", "37", "n/4", "n+5"])
def test_topk_phase_split_form_hops(gpu_session, n, window, hop_of):
    """the split form reads its samples through a buffer descriptor with unaligned 16-B loads for odd
    and overlapping hops; hop = 1, an odd hop (37), N/4 and a gap (N + 5) against the AoS form and the oracle."""
    hop = {"1": 1, "37": 37, "n/4": n // 4, "n+5": n + 5}[hop_of]
    _topk_phase_forms(n, 8, 18, 200, window, hop)


def _topk_phase_forms(n, k, minp, maxp, window, hop):
    torch = pytest.importorskip("torch")
    nwin = 300
    s = synth.random_walk((nwin - 1) * hop + n, seed=n + k + 17 + hop)
    dev = torch.device("cuda", 0)
    d_s = torch.from_numpy(s).to(dev)
    outs = []
    for v in (0, 1):
        plan = bridge.Plan(0, n, hop, nwin, "none", window, output="topk_phase")
        plan.set_topk(k, minp, maxp)
        plan.set_variant(v)
        d_o = torch.full((nwin * 6 * k,), float("nan"), dtype=torch.float64, device=dev)
        plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append(d_o.view(nwin, k, 6).cpu().numpy())
        plan.close()
    # the same scan order and unwrap decisions; not bit-identical, because the AoS form evaluates the cosine windows
    # by rotation and the split form by the three-term recurrence (9e-16 of the window)
    a, b = outs
    same = a[:, :, 0] == b[:, :, 0]
    assert int((~same).sum()) <= 2
    full_max = ref(s, n, hop, "none", window).max(axis=1)[:, None]  # normalised like every parity bar
    assert np.all(np.abs(np.where(same, a[:, :, 1] - b[:, :, 1], 0.0)) <= 1e-13 * full_max)
    got = outs[0]
    want = oracle.batch_topk_phase(s, n, hop, "none", window, 0, None, k, minp, maxp)
    _topk_match(got[:, :, :4], want[:, :, :4], 1e-10, ref(s, n, hop, "none", window).max(axis=1))
    full = oracle.batch_phase(s, n, hop, "none", window)
    for g in outs:
        for w in range(nwin):
            mag = np.sqrt(full[w, 0])
            ok = mag >= 1e-9 * mag.max()
            same = (g[w, :, 0] == want[w, :, 0]) & (want[w, :, 0] >= 0)
            bins = want[w, same, 0].astype(int)
            if ok[: max(bins.max(initial=0), 1) + 2].all():
                assert np.max(np.abs(g[w, same, 4:] - want[w, same, 4:]), initial=0.0) <= 1e-8
            assert np.all(g[w, want[w, :, 0] < 0, 4:] == 0.0)


@pytest.mark.parametrize("length", [2, 6, 64, 1000, 4096, 10002])
@pytest.mark.parametrize("method", ["unwrapped", "wrapped", "group_delay"])
def test_spectral_phase_unwrap(gpu_session, length, method):
    """gpu_spectral_phase_unwrap (L/WaveSpecZZ_1.0.4-core.mq5:72,416) on packed spectra of any even
    length (incl. non-powers of two, as after gpu_spectral_upscale)."""
    rng = np.random.default_rng(length)
    spec = rng.standard_normal(length)
    got = bridge.spectral_phase_unwrap(spec, method)
    ph, u, gd = oracle.phase_unwrap(spec)
    want = {"unwrapped": u, "wrapped": ph, "group_delay": gd}[method]
    assert got.shape == want.shape
    assert np.max(np.abs(got - want)) <= 1e-9


def test_phase_plan_and_bad_precision(gpu_session):
    torch = pytest.importorskip("torch")
    n, w = 2048, 200
    s = synth.random_walk(n * w, seed=8)
    plan = bridge.Plan(0, n, n, w, "none", "blackman", output="phase")
    d_s = torch.from_numpy(s).cuda()
    d_o = torch.empty(w * 3 * (n // 2), dtype=torch.float64, device="cuda")
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = d_o.cpu().numpy().reshape(w, 3, n // 2)
    want = oracle.batch_phase(s, n, n, "none", "blackman")
    assert oracle.rel_err(got[:, 0], want[:, 0]) <= 1e-10
    for i in (0, w // 2, w - 1):
        m = _unwrap_match(got[i, 1], want[i, 1], np.sqrt(want[i, 0]))
        _delay_match(got[i, 2], want[i, 2], np.sqrt(want[i, 0]), m)
    plan.close()
    with pytest.raises(bridge.BridgeError):
        bridge.spectrum_batch(s[: 4 * n], n, n, "none", "hann", 0, "f32", "phase")


@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("nwin,hop", [(1, 256), (63, 256), (65, 256), (130, 256), (200, 1), (150, 37)])
def test_kalman_ragged_and_overlap(gpu_session, prec, nwin, hop):
    """Kalman pre-pass: partial last 64-window tile (range-checked buffer IO), overlapping windows."""
    n = 256
    s = synth.random_walk((nwin - 1) * hop + n, seed=nwin + hop)
    p = gpu(s, n, hop, "kalman", "hann", prec=prec)
    r = ref(s.astype(np.float32).astype(np.float64) if prec == "f32" else s, n, hop, "kalman", "hann")
    assert p.shape == r.shape == (nwin, n // 2)
    assert oracle.rel_err(p, r) <= TOL[prec]


@pytest.mark.parametrize("n,nwin,hop", [(1024, 65, 1024), (2048, 130, 2048), (4096, 63, 4096), (4096, 70, 37),
                                        (8192, 5, 8192), (16384, 9, 16384)])
def test_kalman_f32_two_segments(gpu_session, n, nwin, hop):
    """fp32 Kalman at N >= 1024 with the default flags runs two time segments per lane
    (kalman_pk2_kernel, verified warm-up): parity with the sequential oracle on ragged last tiles
    and overlapping windows, full row and in band."""
    s = synth.random_walk((nwin - 1) * hop + n, seed=n + nwin)
    p = gpu(s, n, hop, "kalman", "hann", prec="f32")
    r = ref(s.astype(np.float32).astype(np.float64), n, hop, "kalman", "hann")
    assert p.shape == r.shape == (nwin, n // 2)
    assert oracle.rel_err(p, r) <= TOL["f32"]
    assert oracle.inband_err(p, r, *oracle.band(n)) <= TOL["f32"]


@pytest.mark.parametrize("kind,seg,at", [("spike", (1,), 0), ("spike", (2,), 0), ("spike", (3,), 0), ("spike", (1, 2, 3), 0),
                                         ("spike", (2,), 128), ("jump", (2,), 0), ("jump", (1,), 200)])
def test_kalman_f32_segments_fallback(gpu_session, kind, seg, at):
    """fp32 Kalman runs time segments that start cold and are verified at the hand-over: the
    library's two-segment kernel (kalman_pk2_kernel) starts its second segment at L0 - WU = 2 S,
    the four-segment ablation (kalman_pk4_kernel) segment k at k S, S = (N + 3 WU)/4 - WU.  A spike of 1000 on a segment's cold-start sample is
    where that segment's reset puts its level: clipped to 6 sigma per step it is still far off
    at the hand-over, so the check against the previous segment's final state must fail and the
    segment be re-run from that state -- for the hand-over across the lane pair (segment 2) and
    for a chain of failures (1, 2, 3) alike.  Unverified, those outputs would be orders of
    magnitude beyond the bar.  Spikes later in the warm-up and level jumps exercise the accepted
    path.  A level jump of 0.5 (an ordinary price gap) is held to the same flat 1e-5: the fp32
    filter re-centres its state on every tile's first sample (kalman_core.h), so the post-jump
    level never sits in the fp32 state (2e-5 -> 1e-6 in scripts/kalman_f32_emulation.py)."""
    n, wu = 4096, 256
    S = (n + 3 * wu) // 4 - wu
    s = synth.random_walk(64 * n, seed=17)
    for w in range(0, 64, 3):  # every third window; the others must take the fast path unharmed
        for k in seg:
            i = w * n + k * S + at
            if kind == "spike":
                s[i] += 1000.0
            else:
                s[i:(w + 1) * n] += 0.5
    s32 = s.astype(np.float32).astype(np.float64)
    p = gpu(s32, n, n, "kalman", "hann", prec="f32")
    r = ref(s32, n, n, "kalman", "hann")
    assert oracle.rel_err(p, r) <= TOL["f32"]
    assert oracle.inband_err(p, r, *oracle.band(n)) <= TOL["f32"]


@pytest.mark.parametrize("n,hop,jump", [(1024, 1024, 0.5), (4096, 4096, -0.5), (4096, 4096, 0.9), (2048, 333, 0.5),
                                        (256, 256, 0.5)])
def test_kalman_f32_level_jumps(gpu_session, n, hop, jump):
    """Level jumps at varied positions (every fourth window, up and down, inside and across tiles,
    overlapping windows) on both fp32 filters (N = 256: sequential kernel; N >= 1024: two
    segments) at the flat fp32 bar, full row and in band."""
    nwin = 48
    s = synth.random_walk((nwin - 1) * hop + n, seed=n + hop)
    rng = np.random.default_rng(n)
    for w in range(0, nwin, 4):
        at = w * hop + int(rng.integers(1, n))
        s[at:] += jump
    s32 = s.astype(np.float32).astype(np.float64)
    p = gpu(s32, n, hop, "kalman", "hann", prec="f32")
    r = ref(s32, n, hop, "kalman", "hann")
    assert oracle.rel_err(p, r) <= TOL["f32"]
    assert oracle.inband_err(p, r, *oracle.band(n)) <= TOL["f32"]


def _kp(**kw):
    names = ["follow", "qp", "qv", "qa", "qj", "adapt", "r", "vp", "vv", "va", "vj", "iv", "ia", "ij", "clip", "ema"]
    p = list(KALMAN)
    for k, v in kw.items():
        p[names.index(k)] = v
    return p


@pytest.mark.parametrize("variant", [1, 2, 7, 8])
def test_kalman_plan_variants(gpu_session, variant):
    """Advisor r05: wsp_plan_set_variant reaches the fp32 Kalman pre-pass of a spectrum plan (it stayed 0 before, so
    the round-5 "variant 7 neutral" A/B timed one kernel twice).  8 = the packed two-segment filter in the original
    basis with the reference's floors (the round-5 default; 0 steps in the Newton basis since round 6); 7 = 8 with its
    rows written through to memory: bit-identical to 8; 1 = single-wave workgroups of the one-lane filter and
    2 = the sequential one-lane filter: other kernels, held to the fp32 bar against the oracle."""
    torch = pytest.importorskip("torch")
    n, nwin = 2048, 700
    s = synth.random_walk(nwin * n, seed=91)
    s.reshape(nwin, n)[::4, n // 3:] += 0.5  # a level jump in every fourth window (trips the clip and the boost)
    dev = torch.device("cuda", 0)
    d_s = torch.from_numpy(s.astype(np.float32)).to(dev)
    outs = []
    for v in (0, variant) + ((8,) if variant == 7 else ()):
        plan = bridge.Plan(0, n, n, nwin, "kalman", "hann", precision="f32")
        plan.set_variant(v)
        d_o = torch.full((nwin * (n // 2),), float("nan"), dtype=torch.float32, device=dev)
        plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append(d_o.view(nwin, n // 2).double().cpu().numpy())
        plan.close()
    base, got = outs[:2]
    if variant == 7:
        assert np.array_equal(got, outs[2])
    # the variant reaches the pre-pass: another kernel rounds differently from the default's Newton basis
    # (round 5's form set no K.variant on the spectrum path, so every variant ran the default kernel)
    assert not np.array_equal(got, base)
    want = ref(s.astype(np.float32).astype(np.float64), n, n, "kalman", "hann")
    assert oracle.rel_err(got, want) <= TOL["f32"]
    assert oracle.rel_err(base, want) <= TOL["f32"]


@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("kw", [dict(ema=20.0), dict(adapt=0.0), dict(clip=0.0), dict(adapt=0.0, clip=0.0, ema=5.0),
                                dict(follow=2.5, iv=1e-4, ia=-1e-6), dict(qp=1e-3, qv=2e-4, qa=5e-5, qj=1e-5),
                                dict(qj=1e-9), dict(r=0.05), dict(vp=1e-3, vv=50.0, va=0.1, vj=3.0, adapt=2.0, clip=3.0)])
def test_kalman_params(gpu_session, prec, kw):
    """gpu_set_kalman_params: non-default flags take the runtime-flag kernel (kalman_kernels.hip); default flags with
    other noise levels take the fp32 two-segment filter in the Newton basis when its floor guard's premises hold
    (slower noise, other initial variances, stronger boost), in the original basis with the floors when they do not
    (q_jerk at its 1e-9 floor: kalman_core.h nb2_ok).  (The measurement noise at its 1e-9 floor is no test case: the trend
    then follows every sample and the detrended windows are rounding noise in both filters.)"""
    kp = _kp(**kw)
    n = 1024
    s = synth.random_walk(70 * n, seed=5)
    bridge.set_kalman_params(kp)
    try:
        p = gpu(s, n, n, "kalman", "hann", prec=prec)
    finally:
        bridge.set_kalman_params(KALMAN)
    s_ref = s.astype(np.float32).astype(np.float64) if prec == "f32" else s
    r = oracle.batch_spectrum(s_ref, n, n, "kalman", "hann", 0, kalman=kp)
    assert oracle.rel_err(p, r) <= TOL[prec], kw


@pytest.mark.parametrize("window", ["hann", "hamming", "blackman", "bartlett", "none"])
@pytest.mark.parametrize("n,nwin,hop", [(1024, 130, 1024), (4096, 70, 4096), (4096, 65, 37), (8192, 9, 8192)])
def test_kalman_window_fold(gpu_session, window, n, nwin, hop):
    """The fp32 two-segment Kalman filter multiplies the plan's window into its rows at N <= 4096 (window pairs staged
    in LDS) and the spectrum launch then takes none; variant 9 keeps the window in the spectrum kernel, and N = 8192
    never folds.  Both against the oracle at the fp32 bar for every window, ragged tiles and overlapping windows
    included, and against each other."""
    torch = pytest.importorskip("torch")
    s = synth.random_walk((nwin - 1) * hop + n, seed=n + nwin + hop)
    dev = torch.device("cuda", 0)
    d_s = torch.from_numpy(s.astype(np.float32)).to(dev)
    outs = []
    for v in (0, 9):
        plan = bridge.Plan(0, n, hop, nwin, "kalman", window, precision="f32")
        plan.set_variant(v)
        d_o = torch.full((nwin * (n // 2),), float("nan"), dtype=torch.float32, device=dev)
        plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append(d_o.view(nwin, n // 2).double().cpu().numpy())
        plan.close()
    want = ref(s.astype(np.float32).astype(np.float64), n, hop, "kalman", window)
    for got in outs:
        assert oracle.rel_err(got, want) <= TOL["f32"], window
        assert oracle.inband_err(got, want, *oracle.band(n)) <= TOL["f32"], window
    assert oracle.rel_err(outs[0], outs[1]) <= 2e-6


def test_kalman_newton_basis_tool_check(gpu_session):
    """The Newton-basis filter's own checks (tools/kalman_bench.hip check, N = 4096, hop 37): its result against the
    fp64 host restatement of StepKalman4D at the fp32 bar with and without forced warm-up re-runs, and with the floor
    guard forced to fail every wave is bit-identical to the original-basis kernel with the reference's floors."""
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parents[1] / "fft-wavespec_amd" / "bin" / "kalman_bench"
    assert exe.exists(), "build() builds bin/kalman_bench"
    out = subprocess.run([str(exe), "check", "4096"], capture_output=True, text=True, timeout=300, check=True).stdout
    lines = [ln for ln in out.splitlines() if "Newton basis" in ln]
    assert len(lines) >= 6, out
    for ln in lines:
        if "max|d-ref|/max|ref|" in ln:
            err = float(ln.split("max|d-ref|/max|ref|")[1].split()[0])
            assert err <= 1e-5, ln
    forced = [ln for ln in lines if "bit-identical to the original-basis kernel" in ln]
    assert len(forced) == 2 and all(ln.rstrip().endswith("yes") for ln in forced), out
    guard = [ln for ln in lines if "guard forced" in ln and "fallback re-runs" in ln]
    assert all("+ 2 guard)" in ln for ln in guard), guard  # W = 100 windows: both waves re-ran


def test_register_host_records_range(gpu_session):
    """gpu_register_host (round 6: the range is recorded, nothing is page-locked, calls stage through the library's
    pinned buffers): a registered fp64 series and output array give results identical to the unregistered path,
    views inside the series are covered, overlapping and unknown ranges are refused."""
    n, hop = 1024, 256
    s = synth.random_walk(300 * hop + n, seed=41)
    nwin = 1 + (s.size - n) // hop
    staged = gpu(s, n, hop, "iir", "hann", 512)
    out = np.full(nwin * (n // 2), np.nan)
    bridge.register_host(s)
    bridge.register_host(out)
    try:
        p = bridge.spectrum_batch(s, n, hop, "iir", "hann", 512, out=out)
        assert p.base is out or p.base is out.base or np.shares_memory(p, out)
        assert np.array_equal(p, staged)
        assert oracle.rel_err(p, ref(s, n, hop, "iir", "hann", 512)) <= TOL["f64"]
        # a view inside the registered series is covered as well (sub-range of the region)
        sub = s[37 * hop:]
        assert oracle.rel_err(gpu(sub, n, hop), ref(sub, n, hop)) <= TOL["f64"]
        # fp32 plans convert and truncated outputs stage: same results as without registration
        p32 = gpu(s, n, hop, "kalman", "hann", prec="f32")
        assert oracle.rel_err(p32, ref(s.astype(np.float32).astype(np.float64), n, hop, "kalman", "hann")) <= TOL["f32"]
        part = bridge.spectrum_batch(s, n, hop, "iir", "hann", 512, max_records=10, out=out)
        assert np.array_equal(part, staged[:10])
        # top-k and the legacy batch FFT take the same path
        tk = bridge.spectrum_topk_batch(s, n, hop)
        w = s[: 8 * n].reshape(8, n).copy()  # its own buffer (a view of s would overlap s)
        bridge.register_host(w)
        fb = bridge.fft_real_forward_batch(w)
        bridge.unregister_host(w)
        assert oracle.rel_err(fb, ref(w.reshape(-1), n, n, "none", "none", output="packed")) <= 1e-12
        assert tk.shape == (nwin, 8, 4)
        # overlapping and unknown ranges are refused
        with pytest.raises(bridge.BridgeError) as e:
            bridge.register_host(s[10:20])
        assert e.value.status == bridge.BAD_ARGS
        with pytest.raises(bridge.BridgeError) as e:
            bridge.unregister_host(s[10:])
        assert e.value.status == bridge.BAD_ARGS
    finally:
        bridge.unregister_host(out)
        bridge.unregister_host(s)
    with pytest.raises(bridge.BridgeError):
        bridge.unregister_host(s)


def test_pinned_feed_cache_grows(gpu_session, tmp_path):
    """FeedCache rewired to pinned buffers: pin_feed_cache registers the chronological history;
    ensure_feed_cache re-registers it when more bars arrive; feed_spectra runs on it in place."""
    n = 512
    hist = synth.random_walk(6000, seed=9)
    close = hist[::-1].copy()  # newest first, as CopyClose fills an as-series array
    cache = indicator.FeedCache()
    ok, _, _ = indicator.ensure_feed_cache(cache, "EURUSD", "M1", 3000, False, "WaveSpecZZ",
                                           lambda start, cnt: close[start:start + cnt], str(tmp_path))
    assert ok and cache.chrono.size == 3000
    indicator.pin_feed_cache(cache)
    try:
        assert cache.pinned
        p = indicator.feed_spectra(cache, n, 64)
        assert oracle.rel_err(p, ref(cache.chrono, n, 64, "none", "hann")) <= TOL["f64"]
        ok, delta, _ = indicator.ensure_feed_cache(cache, "EURUSD", "M1", 6000, False, "WaveSpecZZ",
                                                   lambda start, cnt: close[start:start + cnt], str(tmp_path))
        assert ok and delta == 3000 and cache.pinned and cache.chrono.size == 6000
        assert np.array_equal(cache.chrono, hist)
        p = indicator.feed_spectra(cache, n, 64)
        assert oracle.rel_err(p, ref(hist, n, 64, "none", "hann")) <= TOL["f64"]
    finally:
        indicator.unpin_feed_cache(cache)
    assert not cache.pinned


def _hip_knows(addr: int) -> bool:
    """hipPointerGetAttributes on a host address (the runtime torch loaded, the library's): page-locked?"""
    class Attr(C.Structure):
        _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p),
                    ("hostPointer", C.c_void_p), ("isManaged", C.c_int), ("allocationFlags", C.c_uint)]
    hip = C.CDLL("libamdhip64.so.7")
    a = Attr()
    e = hip.hipPointerGetAttributes(C.byref(a), C.c_void_p(addr))
    hip.hipGetLastError()
    return e == 0 and a.type != 0


def test_register_host_page_edges(gpu_session):
    """Registering buffers that start and end mid-page and share pages with each other and with unregistered memory
    (the round-4 fault layout): the runtime maps none of it (round 6: registration only records the range), the
    batch results equal the staged path's, an overlapping registration is refused, and a buffer with no whole page
    inside registers as well."""
    page = 4096
    n, hop = 512, 7
    arena = np.zeros((16 << 20) // 8)  # one allocation holding several neighbouring arrays
    first = ((37 * 8 - arena.ctypes.data % page) % page) // 8 + page // 8  # 37 doubles past a page start
    s = arena[first:first + 40000]
    s[:] = synth.random_walk(s.size, seed=43)
    nwin = 1 + (s.size - n) // hop
    out = arena[first + 40000:first + 40000 + nwin * (n // 2)]  # starts in s's last page
    assert out.ctypes.data // page == (s.ctypes.data + s.nbytes - 1) // page
    staged = gpu(s.copy(), n, hop, "mean", "hann")
    sid = bridge.session_id()
    assert sid > 0
    bridge.register_host(s)
    bridge.register_host(out)
    try:
        lo = -(-s.ctypes.data // page) * page
        hi = (s.ctypes.data + s.nbytes) // page * page
        assert not _hip_knows(lo) and not _hip_knows(hi - 1)  # recorded only: nothing page-locked
        p = bridge.spectrum_batch(s, n, hop, "mean", "hann", out=out)
        assert np.shares_memory(p, out) and np.array_equal(p, staged)
        sub = s[1001:-333]  # a view that starts and ends mid-page inside the registered range
        assert np.array_equal(gpu(sub, n, hop, "mean", "hann"), gpu(sub.copy(), n, hop, "mean", "hann"))
        with pytest.raises(bridge.BridgeError) as e:
            bridge.register_host(s[5:9])
        assert e.value.status == bridge.BAD_ARGS
        assert bridge.session_id() == sid
    finally:
        bridge.unregister_host(out)
        bridge.unregister_host(s)
    tiny = arena[first + 3:first + 300]
    bridge.register_host(tiny)
    try:
        assert np.array_equal(gpu(tiny, 64, 5), gpu(tiny.copy(), 64, 5))
    finally:
        bridge.unregister_host(tiny)


def test_host_locking_withdrawn(gpu_session):
    """Round 6: page-locking caller memory is withdrawn.  gpu_set_host_locking(1) is refused with
    an explanation, 0 stays the only mode, and a registration made after the refused call page-locks nothing."""
    with pytest.raises(bridge.BridgeError) as e:
        bridge.set_host_locking(1)
    assert e.value.status == bridge.BAD_ARGS and "withdrawn" in str(e.value)
    assert bridge.set_host_locking(0) == 0
    a = np.zeros(1 << 16)
    bridge.register_host(a)
    try:
        assert not _hip_knows(a.ctypes.data + 4096) and not _hip_knows(a.ctypes.data + a.nbytes - 1)
    finally:
        bridge.unregister_host(a)


@pytest.mark.parametrize("case", ["hop1_many_parts", "truncated_mid_part", "f32_kalman", "registered_out"])
def test_sync_ring_copy_out(gpu_session, case):
    """Synchronous batches cut by output bytes (>= 64 MiB parts) and drained through the 4-slot pinned output ring
    (batch_ring_out): an output-dominated hop = 1 batch of ~6 parts (the ring wraps), an out_cap that ends inside a
    part (nothing written past it), an fp32 Kalman batch (converted on the way out) and a registered output array --
    against the device plan of the same batch (one launch, no parts) and, on sampled windows, the oracle."""
    torch = pytest.importorskip("torch")
    n = 2048
    prec, det = ("f32", "kalman") if case == "f32_kalman" else ("f64", "none")
    hop = n if case == "f32_kalman" else 1
    nwin = 4000 if case == "f32_kalman" else 190000  # hop 1: 190000 x 1024 x 8 B = 1.56 GB of records, 24 parts
    s = synth.random_walk((nwin - 1) * hop + n, seed=77)
    rec = n // 2
    out = np.full(nwin * rec, -7.0)
    cap = nwin if case != "truncated_mid_part" else 100000 + 17
    if case == "registered_out":
        bridge.register_host(out)
    try:
        got = bridge.spectrum_batch(s, n, hop, det, "hann", precision=prec, max_records=cap, out=out)
    finally:
        if case == "registered_out":
            bridge.unregister_host(out)
    assert got.shape == (cap, rec)
    if cap < nwin:
        assert (out[cap * rec:] == -7.0).all()
    dev = torch.device("cuda", 0)
    d_s = torch.from_numpy(s.astype(np.float32) if prec == "f32" else s).to(dev)
    plan = bridge.Plan(0, n, hop, nwin, det, "hann", precision=prec)
    d_o = torch.empty(nwin * rec, dtype=torch.float32 if prec == "f32" else torch.float64, device=dev)
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    want = d_o.view(nwin, rec)[:cap].double().cpu().numpy()
    plan.close()
    del d_o, d_s
    if prec == "f64":  # the parts' sliding-DFT segments start at other windows: equal to rounding, not bit for bit
        assert oracle.rel_err(got, want) <= 1e-12
    else:
        assert np.array_equal(got, want)
    rng = np.random.default_rng(5)
    sample = np.unique(np.concatenate([[0, cap - 1], rng.integers(0, cap, 6)]))
    s_ref = s.astype(np.float32).astype(np.float64) if prec == "f32" else s
    for w in sample:
        r = oracle.batch_spectrum(s_ref[w * hop:w * hop + n], n, n, det, "hann", 0, kalman=KALMAN)
        assert oracle.rel_err(got[w:w + 1], r) <= TOL[prec], w


def test_pageable_copies_after_registrations(gpu_session):
    """The round-4 / round-5 fault sequence (profiles/r04/faults, profiles/r05/faults): numpy arrays registered and
    unregistered, freed, and then pageable device-to-host and host-to-device copies through torch into freshly
    allocated host memory of many sizes (the heap then reuses the freed pages) -- every byte must arrive.  With
    page-locking this faulted in the copies (r05diag2, r05final3); in the default mode it must not."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    for r in range(6):
        arrs = [synth.random_walk(m, seed=r * 10 + i) for i, m in enumerate((3000, 8192 + 5, 70001, 300 * 256 + 1024))]
        for a in arrs:
            bridge.register_host(a)
        p = bridge.spectrum_batch(arrs[3], 1024, 256, "none", "hann")
        for a in arrs:
            bridge.unregister_host(a)
        del arrs
        for m in (1 << 10, 3 << 12, 1 << 17, 5 << 18, 1 << 21):
            d = torch.arange(m, dtype=torch.float64, device=dev) + r
            h = d.cpu()
            assert h[-1].item() == m - 1 + r and h[0].item() == r
            back = torch.from_numpy(np.full(m, float(r))).to(dev)
            assert back.sum().item() == r * m
        assert np.isfinite(p).all()
