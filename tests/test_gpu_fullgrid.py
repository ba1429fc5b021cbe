"""Parity at the benchmarked sizes: the exact kernel instantiations bench.py times, on
full-size batches, checked against the oracle on windows sampled from the LAST
grid-stride iterations of each launch (the library launches at most 32768
workgroups and grid-strides: spectrum_dispatch.h kDefaultGrid), plus the in-band
metric over the reference's cycle bins and the worst element-wise error.

Also the 28-symbol C5 fetcher shape from 28 concurrent threads (one per chart,
WaveCyclesBatchFetcher.mq5:104-133) with staggered gpu_shutdown calls.
"""
import ctypes as C
import json
import os
import threading
import time

import numpy as np
import pytest

import oracle
from wavespec_amd import bridge, synth

pytestmark = pytest.mark.gpu

GRID = 32768  # workgroups per launch (spectrum_dispatch.h kDefaultGrid)
KALMAN = oracle.KALMAN_DEFAULTS
METRICS = {}


def _record(name, **kv):
    METRICS[name] = kv
    path = os.environ.get("WSP_PARITY_LOG")
    if path:
        with open(path, "w") as f:
            json.dump(METRICS, f, indent=1)


def _sample(nwin, per_group_windows, k=24, seed=0):
    """Window indices: the first and last windows, a spread, and a block from the last grid-stride
    iteration (w >= (iterations - 1) * GRID * windows-per-workgroup)."""
    rng = np.random.default_rng(seed)
    groups = -(-nwin // per_group_windows)
    iters = -(-groups // GRID)
    last0 = (iters - 1) * GRID * per_group_windows
    tail = np.arange(last0, min(nwin, last0 + 8))
    idx = np.unique(np.r_[0, 1, nwin - 1, nwin - 2, tail, rng.integers(last0, nwin, k // 2),
                          rng.integers(0, nwin, k // 2)])
    return idx, iters


def _numpy_power(X, n):
    """|X_k|^2, k < N/2, of the rows of X with the reference's symmetric Hann, by numpy's FFT on the host (the
    independent check of the full-size tests: device FFT libraries stay out of the GPU test process)."""
    hann = 0.5 * (1 - np.cos(2 * np.pi * np.arange(n) / (n - 1)))
    F = np.fft.rfft(X * hann, axis=1)[:, : n // 2]
    return F.real ** 2 + F.imag ** 2


def _check_power(name, got, want, n, tol):
    kmin, kmax = oracle.band(n)
    full = oracle.rel_err(got, want)
    inb = oracle.inband_err(got, want, kmin, kmax)
    el = oracle.worst_elementwise(got, want, kmin, kmax)
    _record(name, windows=int(got.shape[0]), rel_err=full, inband_err=inb, inband_worst_elementwise=el,
            band=[kmin, kmax])
    assert full <= tol, (name, full)
    assert inb <= tol, (name, inb)
    return el


def test_north_star_full_grid(gpu_session):
    """65536 x 4096 fp64 Hann, no detrend: spectrum_kernel<double,12,none,power,kWinCos> as benchmarked."""
    torch = pytest.importorskip("torch")
    n, w = 4096, 65536
    dev = torch.device("cuda", 0)
    d_s = synth.random_walk_torch(n * w, 11, dev)
    d_o = torch.empty(w * n // 2, dtype=torch.float64, device=dev)
    plan = bridge.Plan(0, n, n, w, "none", "hann")
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    P = d_o.view(w, n // 2)
    assert torch.isfinite(P).all().item() and (P >= 0).all().item()
    idx, iters = _sample(w, 1)
    assert iters == 2 and idx.max() >= GRID
    X = d_s.view(w, n)
    host = X[torch.from_numpy(idx).to(dev)].cpu().numpy()
    got = P[torch.from_numpy(idx).to(dev)].cpu().numpy()
    want = np.stack([oracle.window_spectrum(x, "none", "hann") for x in host])
    el = _check_power("north_star", got, want, n, 1e-10)
    assert el <= 1e-8
    # every 257th window against torch.fft with the reference's symmetric Hann
    hann = 0.5 * (1 - torch.cos(2 * np.pi * torch.arange(n, device=dev, dtype=torch.float64) / (n - 1)))
    F = torch.fft.rfft(X[::257] * hann, dim=1)[:, : n // 2]
    Pt = F.real ** 2 + F.imag ** 2
    err = ((P[::257] - Pt).abs().amax(dim=1) / Pt.abs().amax(dim=1)).max().item()
    assert err < 1e-12
    plan.close()


def test_c3_kalman_f32_full_grid(gpu_session):
    """C3: 65536 x 4096 fp32, per-window Kalman 4D + Hann (pre-pass + spectrum_kernel<float,...>)."""
    torch = pytest.importorskip("torch")
    n, w = 4096, 65536
    dev = torch.device("cuda", 0)
    d_s = synth.random_walk_torch(n * w, 11, dev, torch.float32)
    d_o = torch.empty(w * n // 2, dtype=torch.float32, device=dev)
    plan = bridge.Plan(0, n, n, w, "kalman", "hann", 0, "f32")
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    P = d_o.view(w, n // 2)
    assert torch.isfinite(P).all().item()
    idx, iters = _sample(w, 1, seed=3)
    assert idx.max() >= GRID
    host = d_s.view(w, n)[torch.from_numpy(idx).to(dev)].double().cpu().numpy()
    got = P[torch.from_numpy(idx).to(dev)].double().cpu().numpy()
    want = np.stack([oracle.window_spectrum(x, "kalman", "hann", 0, kalman=KALMAN) for x in host])
    _check_power("c3", got, want, n, 1e-5)
    plan.close()


def test_c3_kalman_f32_full_grid_level_jumps(gpu_session):
    """C3 at full size with a 0.5 level jump (an ordinary price gap) inside every fourth window,
    at a position that varies per window: the fp32 filter's per-tile re-centring keeps it at the
    flat fp32 bar (1e-5, full row and in band)."""
    torch = pytest.importorskip("torch")
    n, w = 4096, 65536
    dev = torch.device("cuda", 0)
    d_s = synth.random_walk_torch(n * w, 11, dev, torch.float64)
    X = d_s.view(w, n)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    at = torch.randint(1, n, (w // 4,), generator=g, device=dev)
    cols = torch.arange(n, device=dev)
    X[::4] += 0.5 * (cols[None, :] >= at[:, None]).double()
    d_s = d_s.float()
    d_o = torch.empty(w * n // 2, dtype=torch.float32, device=dev)
    plan = bridge.Plan(0, n, n, w, "kalman", "hann", 0, "f32")
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    P = d_o.view(w, n // 2)
    assert torch.isfinite(P).all().item()
    idx, _ = _sample(w, 1, k=32, seed=6)
    idx = np.unique(np.r_[idx, idx - idx % 4, np.arange(w - 64, w, 4)])  # jump windows included
    host = d_s.view(w, n)[torch.from_numpy(idx).to(dev)].double().cpu().numpy()
    got = P[torch.from_numpy(idx).to(dev)].double().cpu().numpy()
    want = np.stack([oracle.window_spectrum(x, "kalman", "hann", 0, kalman=KALMAN) for x in host])
    _check_power("c3_level_jumps", got, want, n, 1e-5)
    plan.close()


def test_c4_hop1_full_grid(gpu_session):
    """C4: 1,048,576 overlapping 2048-pt windows, hop = 1, fp64 Hann (8 GiB of spectra in HBM), as
    benchmarked: the default algorithm takes the seeded sliding DFT (sliding_dft.hip), whose
    workgroups each seed one segment of consecutive windows with in-LDS FFTs and slide the rest.
    Sampled: both ends, a spread, and the windows either side of segment seams (first and last
    window of a segment: the seed and the longest slide) for every segment length the library
    picks (32 ... 256, a power of two); the whole batch is checked against the FFT kernel window
    by window in tests/test_gpu_slide.py::test_slide_vs_fft_large_segments."""
    torch = pytest.importorskip("torch")
    n, w = 2048, 1048576
    dev = torch.device("cuda", 0)
    d_s = synth.random_walk_torch(w - 1 + n, 13, dev)
    d_o = torch.empty(w * (n // 2), dtype=torch.float64, device=dev)
    plan = bridge.Plan(0, n, 1, w, "none", "hann")
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    P = d_o.view(w, n // 2)
    rng = np.random.default_rng(4)
    seams = np.concatenate([[k * seg - 1, k * seg] for seg in (32, 64, 128, 256)
                            for k in rng.integers(1, w // seg, 4)])
    idx = np.unique(np.r_[0, 1, w - 2, w - 1, np.arange(w - 300, w, 37), rng.integers(0, w, 16), seams])
    s = d_s.cpu().numpy()
    got = P[torch.from_numpy(idx).to(dev)].cpu().numpy()
    want = np.stack([oracle.window_spectrum(s[i:i + n], "none", "hann") for i in idx])
    el = _check_power("c4", got, want, n, 1e-10)
    assert el <= 1e-8
    assert torch.isfinite(P[-65536:]).all().item()
    del d_o
    plan.close()


@pytest.mark.parametrize("output", ["topk", "topk_phase"])
def test_ns_topk_full_grid(gpu_session, output):
    """North star -> top-8 bins in periods [18, 200] (the benchmarked ns_topk / ns_topk_phase kernels)."""
    torch = pytest.importorskip("torch")
    n, w, k = 4096, 65536, 8
    rw = 4 if output == "topk" else 6
    dev = torch.device("cuda", 0)
    d_s = synth.random_walk_torch(n * w, 11, dev)
    d_o = torch.empty(w * rw * k, dtype=torch.float64, device=dev)
    plan = bridge.Plan(0, n, n, w, "none", "hann", output=output)
    plan.set_topk(k, 18.0, 200.0)
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    R = d_o.view(w, k, rw)
    idx, _ = _sample(w, 1, seed=5)
    host = d_s.view(w, n)[torch.from_numpy(idx).to(dev)].cpu().numpy()
    got = R[torch.from_numpy(idx).to(dev)].cpu().numpy()
    f = oracle.batch_topk if output == "topk" else oracle.batch_topk_phase
    want = np.concatenate([f(x, n, n, "none", "hann", 0, None, k, 18.0, 200.0) for x in host])
    spec = np.stack([oracle.window_spectrum(x, "none", "hann") for x in host])
    kmin, kmax = oracle.band(n)
    band_max = spec[:, kmin:kmax + 1].max(axis=1)
    nb = 0
    for i in range(len(idx)):
        same = got[i, :, 0] == want[i, :, 0]
        nb += int((~same).sum())
        # powers of every slot within 1e-10 of the in-band maximum (rank swaps only between near-ties)
        assert np.max(np.abs(got[i, :, 1] - want[i, :, 1])) <= 1e-10 * band_max[i], i
        if output == "topk_phase":
            assert np.max(np.abs(got[i, same, 4:] - want[i, same, 4:]), initial=0.0) <= 1e-8, i
    assert nb <= 2  # a swap needs two powers equal to ~1e-10: essentially never
    _record(f"ns_{output}", windows=len(idx), bin_mismatches=nb)
    plan.close()


@pytest.mark.parametrize("data", ["c4", "noise"])
def test_c4_topk_probe_scan_vs_oracle_full_size(gpu_session, data):
    """The benchmarked hop = 1 top-8 scan (c4_topk: 1,048,576 windows x 2048, the default probe-threshold kernel,
    L/WaveSpecZZ_1.0.3-pla-kalman-fast-gpuopt-nodetrend.mq5:536-554) against the oracle's ora_batch_topk at full
    size, on windows sampled where the scan's paths meet: both ends of the batch, the segment seams (every
    segment start the policy chose, with the window before it and the first window of the next staged batch),
    every window where more candidates passed the threshold than the list holds (the exact-scan fallback,
    flagged by the kernel through wsp_plan_set_scan_flags), and a random spread.  Records the fallback rate.  On C4's
    random walk the fallback never fires (the probe threshold admits 8.4 candidates per window on average); white noise
    (flat band: the winners change every few windows) drives it at scale."""
    torch = pytest.importorskip("torch")
    n, nwin, k = 2048, 1_048_576, 8
    dev = torch.device("cuda", 0)
    if data == "c4":
        d_s = synth.random_walk_torch(nwin + n - 1, 13, dev)
    else:
        g = torch.Generator(device=dev)
        g.manual_seed(29)
        d_s = 1.1 + 1e-3 * torch.randn(nwin + n - 1, dtype=torch.float64, device=dev, generator=g)
    plan = bridge.Plan(0, n, 1, nwin, "none", "hann", output="topk")
    plan.set_topk(k, 18.0, 200.0)
    assert plan.algorithm() == "slide"
    d_o = torch.empty(nwin * 4 * k, dtype=torch.float64, device=dev)
    flags = torch.full((nwin,), 255, dtype=torch.uint8, device=dev)
    plan.set_scan_flags(flags.data_ptr())
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    # the records without the diagnostics are the same
    d_o2 = torch.empty_like(d_o)
    plan.set_scan_flags(0)
    plan.execute(d_s.data_ptr(), d_o2.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(d_o, d_o2)
    del d_o2
    f = flags.cpu().numpy()
    assert f.max() <= 2, "every window reports its path"
    starts = np.flatnonzero(f == 1)
    over = np.flatnonzero(f == 2)
    seg = np.diff(starts)
    assert starts[0] == 0 and len(starts) >= 1
    rng = np.random.default_rng(4)
    seams = starts[1:] if len(starts) <= 600 else rng.choice(starts[1:], 600, replace=False)
    over_s = over if len(over) <= 3000 else rng.choice(over, 3000, replace=False)
    idx = np.unique(np.r_[np.arange(64), np.arange(nwin - 64, nwin), seams - 1, seams, seams + 16, over_s,
                          rng.integers(0, nwin, 2000)])
    idx = idx[(idx >= 0) & (idx < nwin)]
    host = d_s.cpu().numpy()
    R = d_o.view(nwin, k, 4)
    got = R[torch.from_numpy(idx).to(dev)].cpu().numpy()
    want = np.concatenate([oracle.batch_topk(host[i:i + n], n, 1, "none", "hann", 0, None, k, 18.0, 200.0)
                           for i in idx])
    kmin, kmax = oracle.band(n)
    band_max = np.array([oracle.window_spectrum(host[i:i + n], "none", "hann")[kmin:kmax + 1].max() for i in idx])
    same = got[:, :, 0] == want[:, :, 0]
    _record(f"c4_topk_full_size_{data}", windows_checked=int(len(idx)), segments=int(len(starts)),
            segment_lengths=sorted({int(x) for x in seg}) + [int(nwin - starts[-1])],
            fallback_windows=int(len(over)), fallback_rate=float(len(over) / nwin),
            checked_fallbacks=int(len(over_s)), bin_mismatches=int((~same).sum()))
    print(f"c4_topk ({data}): {len(starts)} segments, {len(over)} overflow fallbacks ({len(over) / nwin:.2e} of windows), "
          f"{len(idx)} windows checked, {int((~same).sum())} rank swaps")
    from test_gpu_slide import _topk_bars
    _topk_bars(got, want, band_max, max_swaps=8)
    del d_o
    plan.close()


# ------------------------------------------------------------------ C5 concurrency
def _fetcher(sym, n, series, res, barrier_a, barrier_b, early):
    """WaveCyclesBatchFetcher::OnTimer (WaveCyclesBatchFetcher.mq5:104-133) on the spectrum batch API:
    gpu_init -> submit(hop 1) -> poll try_get with Sleep(5) -> gpu_free_job; then the chart's
    OnDeinit gpu_shutdown (1.1.0:710-716), either right away (early) or after a second round."""
    lib = bridge.lib()
    try:
        assert lib.gpu_init(0, 64) == bridge.OK

        def one_round():
            nwin = series.size - n + 1
            out = np.empty((nwin, n // 2))
            jid = C.c_int64(0)
            st = lib.gpu_submit_spectrum_batch(bridge._dptr(series), series.size, n, 1, 0, 1, 0, 0, 0, C.byref(jid))
            assert st == bridge.OK and jid.value > 0, st
            ready, got = C.c_int32(0), C.c_int32(0)
            # WaveCyclesBatchFetcher.mq5:126-132 verbatim: 4000 tries, Sleep(5) only on OK && ready == 0,
            # break on any status other than OK / NOT_READY (NOT_READY would re-poll at once)
            tries, st = 0, bridge.OK
            while tries < 4000 and ready.value == 0:
                st = lib.gpu_try_get_spectrum_batch(jid.value, bridge._dptr(out), out.size, C.byref(got),
                                                    C.byref(ready))
                if st == bridge.OK and ready.value == 0:
                    time.sleep(0.005)
                elif st != bridge.OK and st != bridge.NOT_READY:
                    break
                tries += 1
            assert st == bridge.OK and ready.value == 1 and got.value == nwin, (st, ready.value, got.value, tries)
            assert lib.gpu_free_job(jid.value) == bridge.OK
            return out

        out1 = one_round()
        barrier_a.wait(timeout=600)
        if early:
            lib.gpu_shutdown()  # this chart closes while the others still work
            barrier_b.wait(timeout=600)
            res[sym] = (out1, None)
            return
        barrier_b.wait(timeout=600)  # every early chart has shut down
        out2 = one_round()  # the session is still open for the charts that did not shut down
        lib.gpu_shutdown()
        res[sym] = (out1, out2)
    except BaseException as e:  # noqa: BLE001 -- reported by the main thread
        res[sym] = e
        barrier_a.abort()
        barrier_b.abort()


def test_c5_28_symbols_concurrent(gpu_session):
    """C5: 28 symbols x 20000 bars, N = 512/1024/2048/4096 (7 symbols each), hop = 1, fp64 Hann,
    from 28 threads at once; half the charts shut down while the other half keep submitting."""
    bars, lens = 20000, (512, 1024, 2048, 4096)
    series = [synth.random_walk(bars, 100 + s) for s in range(28)]
    res = {}
    ba, bb = threading.Barrier(28), threading.Barrier(28)
    th = [threading.Thread(target=_fetcher, args=(s, lens[s // 7], series[s], res, ba, bb, s % 2 == 0))
          for s in range(28)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=900)
    errs = {s: r for s, r in res.items() if isinstance(r, BaseException)}
    assert not errs, errs
    assert len(res) == 28
    worst = 0.0
    for s in range(28):
        n = lens[s // 7]
        nwin = bars - n + 1
        idx = np.unique(np.r_[0, nwin // 2, nwin - 1, np.random.default_rng(s).integers(0, nwin, 3)])
        want = np.stack([oracle.window_spectrum(series[s][i:i + n], "none", "hann") for i in idx])
        for out in res[s]:
            if out is None:
                continue
            assert oracle.rel_err(out[idx], want) <= 1e-10, s
            assert oracle.inband_err(out[idx], want, *oracle.band(n)) <= 1e-10, s
            worst = max(worst, oracle.rel_err(out[idx], want))
    _record("c5_threads", symbols=28, rel_err=worst)
    # the fixture's own reference still holds the session
    s = synth.random_walk(8 * 512, seed=1)
    assert oracle.rel_err(bridge.spectrum_batch(s, 512, 512), oracle.batch_spectrum(s, 512, 512)) <= 1e-10


def test_c5_grouped_plan(gpu_session):
    """C5 as benchmarked (bench.py --config c5): one grouped device plan over the 28 symbols
    (wsp_group_*: one mixed-length persistent sliding-DFT launch).  Every symbol's
    sampled windows -- both ends, a spread, and windows either side of the segment seams of every
    segment length the launcher may pick -- against the oracle (1e-10 full row and in band); the
    whole of every symbol's output against its own single-symbol plan (1e-10)."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    bars, lens = 20000, (512, 1024, 2048, 4096)
    nwins = [bars - lens[s // 7] + 1 for s in range(28)]
    series = [synth.random_walk_torch(bars, 100 + s, dev) for s in range(28)]
    outs = [torch.full((nwins[s] * (lens[s // 7] // 2),), float("nan"), dtype=torch.float64, device=dev)
            for s in range(28)]
    g = bridge.Group(0, [lens[s // 7] for s in range(28)], nwins)
    assert g.launches == 1  # the mixed-length persistent launch (slide_mixed.hip)
    assert g.algorithmic_bytes == sum((bars + nwins[s] * (lens[s // 7] // 2)) * 8 for s in range(28))
    g.execute([x.data_ptr() for x in series], [o.data_ptr() for o in outs], torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    worst = 0.0
    rng = np.random.default_rng(8)
    for s in range(28):
        n, nw = lens[s // 7], nwins[s]
        P = outs[s].view(nw, n // 2)
        assert torch.isfinite(P).all().item()
        # seams of the per-length policy's lengths, and of the mixed launch's (~two tasks per resident workgroup:
        # 459.6M bins / (2 x 512 x 2048) = 220 windows at 512 resident workgroups)
        seams = np.concatenate([[k * sg - 1, k * sg] for sg in (32, 64, 128, 256, *range(100, 121), *range(200, 241)) for k in (1, nw // sg)])
        idx = np.unique(np.clip(np.r_[0, 1, nw - 2, nw - 1, rng.integers(0, nw, 6), seams], 0, nw - 1))
        x = series[s].cpu().numpy()
        want = np.stack([oracle.window_spectrum(x[i:i + n], "none", "hann") for i in idx])
        got = P[torch.from_numpy(idx).to(dev)].cpu().numpy()
        assert oracle.rel_err(got, want) <= 1e-10, s
        assert oracle.inband_err(got, want, *oracle.band(n)) <= 1e-10, s
        worst = max(worst, oracle.rel_err(got, want))
        plan = bridge.Plan(0, n, 1, nw, "none", "hann")
        ref = torch.empty_like(outs[s])
        plan.execute(series[s].data_ptr(), ref.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        Q = ref.view(nw, n // 2)
        rel = ((P - Q).abs().amax(dim=1) / Q.abs().amax(dim=1)).max().item()
        assert rel <= 1e-10, (s, rel)
        plan.close()
    _record("c5_group", symbols=28, rel_err=worst)
    g.close()


def test_c2_full_size(gpu_session):
    """C2 at its benchmarked size (4096 x 1024, hop = 1024, fp64 Hann: spectrum_kernel<double,10,...>, one
    grid-stride iteration): every window against numpy's FFT on the host with the reference's symmetric Hann,
    and sampled windows against the oracle."""
    torch = pytest.importorskip("torch")
    n, w = 1024, 4096
    dev = torch.device("cuda", 0)
    d_s = synth.random_walk_torch(n * w, 17, dev)
    d_o = torch.empty(w * n // 2, dtype=torch.float64, device=dev)
    plan = bridge.Plan(0, n, n, w, "none", "hann")
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    P = d_o.view(w, n // 2).cpu().numpy()
    X = d_s.view(w, n).cpu().numpy()
    Pt = _numpy_power(X, n)
    err = (np.abs(P - Pt).max(axis=1) / np.abs(Pt).max(axis=1)).max()
    assert err < 1e-12, err
    idx, _ = _sample(w, 2, seed=9)
    host, got = X[idx], P[idx]
    want = np.stack([oracle.window_spectrum(x, "none", "hann") for x in host])
    _check_power("c2", got, want, n, 1e-10)
    plan.close()


@pytest.mark.parametrize("n,w", [(65536, 4096), (131072, 2048), (262144, 1024)])
def test_large_full_batches(gpu_session, n, w):
    """The benchmarked large-N batches through the default forms (fused one-workgroup-per-window kernel at
    N = 65536; two passes at N = 131072 and at N = 262144 with 8-column column workgroups and the XCD-aware row
    order there): every
    window against numpy's FFT on the host with the symmetric Hann (max error relative to the window's largest
    bin), and the first, last and two middle windows -- one of them in the last chunk -- against the oracle."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    d_s = synth.random_walk_torch(n * w, 23, dev)
    d_o = torch.empty(w * (n // 2), dtype=torch.float64, device=dev)
    plan = bridge.Plan(0, n, n, w, "none", "hann")
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    P = d_o.view(w, n // 2).cpu().numpy()
    X = d_s.view(w, n).cpu().numpy()
    del d_o, d_s
    err = 0.0
    for c0 in range(0, w, 64):
        Pt = _numpy_power(X[c0:c0 + 64], n)
        err = max(err, (np.abs(P[c0:c0 + 64] - Pt).max(axis=1) / np.abs(Pt).max(axis=1)).max())
    assert err < 1e-11, err
    idx = np.array([0, w // 3, w - 37, w - 1])
    host, got = X[idx], P[idx]
    want = np.stack([oracle.window_spectrum(x, "none", "hann") for x in host])
    _check_power(f"large_{n}", got, want, n, 1e-10)
    _record(f"large_{n}_vs_torch", windows=w, max_rel_err=err)
    plan.close()


def test_ns_phase_full_grid(gpu_session):
    """The benchmarked phase record (ns_phase: 65536 x 4096 fp64 Hann -> [P | unwrapped phase | group delay]):
    sampled windows from both grid-stride iterations against the oracle with the parity suite's near-tie
    conditioning of the unwrap decisions."""
    torch = pytest.importorskip("torch")
    from test_gpu_parity import _delay_match, _unwrap_match
    n, w = 4096, 65536
    dev = torch.device("cuda", 0)
    d_s = synth.random_walk_torch(n * w, 29, dev)
    d_o = torch.empty(w * 3 * (n // 2), dtype=torch.float64, device=dev)
    plan = bridge.Plan(0, n, n, w, "none", "hann", output="phase")
    plan.execute(d_s.data_ptr(), d_o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    R = d_o.view(w, 3, n // 2)
    idx, iters = _sample(w, 1, k=12, seed=31)
    assert iters == 2
    host = d_s.view(w, n)[torch.from_numpy(idx).to(dev)].cpu().numpy()
    got = R[torch.from_numpy(idx).to(dev)].cpu().numpy()
    want = np.concatenate([oracle.batch_phase(x, n, n, "none", "hann") for x in host])
    assert oracle.rel_err(got[:, 0], want[:, 0]) <= 1e-10
    for i in range(len(idx)):
        mag = np.sqrt(want[i, 0])
        m = _unwrap_match(got[i, 1], want[i, 1], mag)
        _delay_match(got[i, 2], want[i, 2], mag, m)
    _record("ns_phase", windows=len(idx))
    plan.close()
