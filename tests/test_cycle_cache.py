"""Cycle-cache file formats (wavespec_amd.cycle_cache).

Byte layouts are checked against the reference's writers
(WaveSpecZZ_1.1.0-gpuopt.mq5:287-324, WaveCyclesBatchFetcher.mq5:59-89);
the warmup reconstruction against a literal per-bar transliteration of
1.1.0:1066-1099 on small cases.  No GPU.
"""
import math
import struct

import numpy as np
import pytest

from wavespec_amd import cycle_cache as cc


def test_name_matches_reference_format():
    assert cc.cycle_cache_name("EURUSD", "PERIOD_M1", 4096, 1, 10, 4) == "WaveSpecZZ_cycles_EURUSD_PERIOD_M1_w4096_m1_ar10_k4.bin"


def test_indicator_round_trip_and_layout(tmp_path):
    rng = np.random.default_rng(1)
    buf = rng.standard_normal((7, 20))
    p = tmp_path / "c.bin"
    cc.save_cycle_cache(str(p), buf)
    raw = p.read_bytes()
    assert struct.unpack("<iii", raw[:12]) == (1, 7, 2)
    assert len(raw) == 12 + 7 * 20 * 8
    # bar 3, field PhaseVal2 (index 7) at byte 12 + 8 * (3 * 20 + 7)
    assert struct.unpack_from("<d", raw, 12 + 8 * (3 * 20 + 7))[0] == buf[3, 7]
    np.testing.assert_array_equal(cc.load_cycle_cache(str(p), 100), buf)
    np.testing.assert_array_equal(cc.load_cycle_cache(str(p), 4), buf[:4])  # count = min(bars, rates_total)


def test_loader_rejections(tmp_path):
    p = tmp_path / "c.bin"
    assert cc.load_cycle_cache(str(p), 10) is None  # no file
    for head in [(2, 3, 2), (1, 3, 0), (1, 3, 3)]:  # version != 1, topk outside [1, 2] (1.1.0:238-241)
        p.write_bytes(struct.pack("<iii", *head) + b"\0" * 8 * 60)
        assert cc.load_cycle_cache(str(p), 10) is None
    p.write_bytes(struct.pack("<iii", 1, 3, 1) + struct.pack("<3d", 1.0, 2.0, 3.0))  # short body: zeros past EOF
    got = cc.load_cycle_cache(str(p), 10)
    assert got.shape == (3, 20) and list(got[0, :3]) == [1.0, 2.0, 3.0] and not got[0, 3:].any() and not got[1:].any()


def _records(n, stride=15, seed=2, method=1):
    rng = np.random.default_rng(seed)
    c = rng.uniform(0.1, 1.0, (n, stride))
    c[:, 1] = rng.uniform(0.01, 0.05, n)   # freq (cycles per bar)
    c[:, 2] = 1.0 / c[:, 1]                 # period
    c[:, 3] = rng.uniform(-3, 3, n)         # phase
    c[:, 5] = rng.uniform(0, 3000, n)       # eta seconds
    c[:, 8] = rng.uniform(-10, 20, n)       # snr dB
    c[:, 14] = method
    return c


def test_fetcher_layout(tmp_path):
    c = _records(6)
    p = tmp_path / "f.bin"
    cc.save_fetcher_cycle_cache(str(p), c.reshape(-1), out_len=6, stride=15, bars=500, top_k=4)
    raw = p.read_bytes()
    assert struct.unpack("<iii", raw[:12]) == (1, 500, 2)  # bars = prices, topk = min(InpTopK, 2)
    assert len(raw) == 12 + 6 * 11 * 8
    rec = np.frombuffer(raw[12:], "<f8").reshape(6, 11)
    np.testing.assert_array_equal(rec, c[:, [0, 1, 2, 3, 5, 6, 7, 8, 10, 11, 13]])
    bars, topk, back = cc.read_fetcher_cycle_cache(str(p))
    assert (bars, topk) == (500, 2)
    np.testing.assert_array_equal(back, rec)


def test_indicator_reads_fetcher_file_as_the_reference_does(tmp_path):
    """The mismatch: LoadCycleCache takes the fetcher's 11-double cycle records as 20-double bars."""
    c = _records(8)
    p = tmp_path / "f.bin"
    cc.save_fetcher_cycle_cache(str(p), c.reshape(-1), 8, 15, bars=30, top_k=2)
    got = cc.load_cycle_cache(str(p), 30)
    flat = c[:, [0, 1, 2, 3, 5, 6, 7, 8, 10, 11, 13]].reshape(-1)  # 88 doubles in the file
    assert got.shape == (30, 20)
    np.testing.assert_array_equal(got.reshape(-1)[:88], flat)
    assert not got.reshape(-1)[88:].any()


def _warmup_literal(cycles, out_len, stride, top_k, hop, n, got, psec, music_only=True, use_weights=True,
                    min_coher=0.05, min_score=0.01, min_snr=-40.0):
    """Line-by-line 1.1.0:1066-1099."""
    B = np.full((got, 20), cc.EMPTY_VALUE)
    two_pi = 6.28318530717958647692
    for c in range(out_len):
        base = c * stride
        method_id = int(cycles[base + 14]) if stride > 14 else 0
        if music_only and method_id != 1:
            continue
        amp, freq, period, phase = cycles[base + 0], cycles[base + 1], cycles[base + 2], cycles[base + 3]
        eta_sec = cycles[base + 5]
        energy, coher, snr = cycles[base + 6], cycles[base + 7], cycles[base + 8]
        eigen, score, etac = cycles[base + 10], cycles[base + 11], cycles[base + 13]
        w_energy, w_coher, w_score = max(energy, 0.0), max(coher, 0.0), max(score, 0.0)
        snr_eff = max(snr, min_snr)
        w_snr = 1.0 / (1.0 + math.pow(10.0, -snr_eff / 10.0))
        wt = (w_energy * w_coher * w_score * w_snr) if use_weights else 1.0
        if coher < min_coher or score < min_score:
            wt = 0.0
        start_bar = (c // top_k) * hop
        if start_bar >= got:
            continue
        omega = two_pi * freq
        span = min(n - 1, got - start_bar - 1)
        slot = c % top_k
        off = 0 if slot == 0 else 1
        for k in range(span + 1):
            idx = start_bar + k
            theta = phase - omega * k
            row = [amp * wt * math.sin(theta), period, max(eta_sec - k * psec, 0.0), theta, energy, coher, snr, score,
                   eigen, etac]
            for j, v in enumerate(row):
                B[idx, 2 * j + off] = v
    return B


@pytest.mark.parametrize("top_k,hop,n,got", [(2, 1, 16, 40), (4, 3, 8, 25), (1, 5, 12, 12)])
def test_warmup_reconstruction(top_k, hop, n, got):
    nwin = 1 + (got - n) // hop
    out_len = nwin * top_k
    c = _records(out_len, seed=top_k + hop)
    c[::3, 14] = 0  # FFT-ridge records: dropped under InpMusicOnly
    c[1::5, 7] = 0.01  # below InpMinCoherence: weight 0
    flat = c.reshape(-1)
    for music_only in (True, False):
        ref = _warmup_literal(flat, out_len, 15, top_k, hop, n, got, 60, music_only=music_only)
        got_b = cc.warmup_buffers(flat, out_len, 15, top_k, hop, n, got, 60, music_only=music_only)
        np.testing.assert_array_equal(got_b, ref)


def test_fetcher_to_indicator_round_trip(tmp_path):
    top_k, hop, n, got = 2, 1, 16, 40
    out_len = (1 + (got - n) // hop) * top_k
    c = _records(out_len)
    fp, ip = tmp_path / "f.bin", tmp_path / "i.bin"
    cc.save_fetcher_cycle_cache(str(fp), c.reshape(-1), out_len, 15, got, top_k)
    buf = cc.fetcher_to_indicator(str(fp), str(ip), top_k, hop, n, 60, method=1)
    # fields the fetcher dropped (eta_bars, residual, kalman_pred) do not enter the buffers
    ref = _warmup_literal(c.reshape(-1), out_len, 15, top_k, hop, n, got, 60)
    np.testing.assert_array_equal(buf, ref)
    np.testing.assert_array_equal(cc.load_cycle_cache(str(ip), got), ref)
