"""Cycle-cache files of WaveSpecZZ.

Two writers in the reference produce files of the same name with different
layouts:

* the indicator (WaveSpecZZ_1.1.0-gpuopt.mq5:224-324, LoadCycleCache /
  SaveCycleCache): int32 version = 1, int32 bars, int32 topk (always 2 when
  written), then per bar 20 doubles -- the per-bar plot buffers of the two
  reconstructed waves (:301-320 order, :INDICATOR_FIELDS);
* WaveCyclesBatchFetcher.mq5:59-89: the same header (bars = the number of
  prices, topk = min(InpTopK, 2)) followed by one 11-double record per cycle
  returned by gpu_try_get_cycles_batch (fields 0,1,2,3,5,6,7,8,10,11,13 of
  the 15-double stride, :FETCHER_FIELDS) -- not per bar, and without the
  method id, ETA in bars, residual power and Kalman prediction.

The indicator's loader reads a fetcher file as 20 doubles per bar from the
cycle records (the mismatch the survey names); :func:`load_cycle_cache`
reproduces that reading exactly (reads past the end of the file give 0.0,
the value MQL5's FileReadDouble returns at end of file).
:func:`fetcher_to_indicator` is the build's conversion: it rebuilds the
15-double records from a fetcher file and replays the batch-warmup
reconstruction of 1.1.0:1066-1099 (:func:`warmup_buffers`) to write a file
the indicator loads as intended.

All integers and doubles are little-endian (MQL5 FileWriteInteger(INT_VALUE)
/ FileWriteDouble on x86).
"""
from __future__ import annotations

import math
import os
import struct

import numpy as np

EMPTY_VALUE = np.finfo(np.float64).max  # MQL5 EMPTY_VALUE == DBL_MAX

# per-bar buffer order of SaveCycleCache / LoadCycleCache (1.1.0:260-279, 301-320)
INDICATOR_FIELDS = (
    "WaveBuffer1", "WaveBuffer2", "WavePeriod1", "WavePeriod2", "EtaCount1", "EtaCount2", "PhaseVal1", "PhaseVal2",
    "MusEnergy1", "MusEnergy2", "MusCoher1", "MusCoher2", "MusSnrDb1", "MusSnrDb2", "MusScore1", "MusScore2",
    "MusEigen1", "MusEigen2", "MusEtaConf1", "MusEtaConf2",
)
# gpu_extract_cycles record (stride 15; field list at 1.1.0:330)
CYCLE_RECORD = (
    "amplitude", "freq", "period", "phase", "eta_bars", "eta_seconds", "energy_ratio", "coherence", "snr_db",
    "residual_power", "eigen_ratio", "score", "kalman_pred", "eta_confidence", "method",
)
# record fields the fetcher writes, in file order (WaveCyclesBatchFetcher.mq5:75-85)
FETCHER_FIELDS = (0, 1, 2, 3, 5, 6, 7, 8, 10, 11, 13)

_HEAD = struct.Struct("<iii")


def cycle_cache_name(symbol: str, tf: str, fft_window: int, method: int, ar_order: int, top_k: int) -> str:
    """CycleCacheName (1.1.0:224-229; the fetcher's copy WaveCyclesBatchFetcher.mq5:51-57
    formats its own inputs InpSymbol/InpTF/InpMethod/InpArOrder/InpTopK the same way)."""
    return f"WaveSpecZZ_cycles_{symbol}_{tf}_w{fft_window}_m{method}_ar{ar_order}_k{top_k}.bin"


def save_cycle_cache(path: str, buffers: np.ndarray) -> None:
    """SaveCycleCache(bars) (1.1.0:287-324): header (1, bars, 2), then 20 doubles per bar.

    ``buffers`` is (bars, 20) in INDICATOR_FIELDS order.
    """
    b = np.ascontiguousarray(buffers, dtype="<f8")
    if b.ndim != 2 or b.shape[1] != len(INDICATOR_FIELDS):
        raise ValueError(f"buffers must be (bars, {len(INDICATOR_FIELDS)})")
    with open(path, "wb") as f:
        f.write(_HEAD.pack(1, b.shape[0], 2))
        f.write(b.tobytes())


def load_cycle_cache(path: str, rates_total: int) -> np.ndarray | None:
    """LoadCycleCache(rates_total) (1.1.0:231-285).

    Returns (count, 20) with count = min(bars, rates_total), or None where the
    reference returns false (no file, version != 1, topk outside [1, 2]).
    Doubles past the end of the file read as 0.0.
    """
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < _HEAD.size:
        return None
    version, bars, topk = _HEAD.unpack_from(data)
    if version != 1 or topk < 1 or topk > 2:
        return None
    count = max(0, min(bars, rates_total))
    want = count * len(INDICATOR_FIELDS)
    body = np.frombuffer(data, dtype="<f8", count=min(want, (len(data) - _HEAD.size) // 8), offset=_HEAD.size)
    out = np.zeros(want)
    out[:body.size] = body
    return out.reshape(count, len(INDICATOR_FIELDS))


def save_fetcher_cycle_cache(path: str, cycles: np.ndarray, out_len: int, stride: int, bars: int, top_k: int) -> None:
    """WaveCyclesBatchFetcher SaveCycleCache (WaveCyclesBatchFetcher.mq5:59-89)."""
    c = np.asarray(cycles, dtype=np.float64).reshape(-1)
    if stride < 14 or out_len * stride > c.size:
        raise ValueError("cycles too short for out_len records of this stride")
    rec = c[: out_len * stride].reshape(out_len, stride)[:, FETCHER_FIELDS]
    with open(path, "wb") as f:
        f.write(_HEAD.pack(1, bars, min(top_k, 2)))
        f.write(np.ascontiguousarray(rec, dtype="<f8").tobytes())


def read_fetcher_cycle_cache(path: str) -> tuple[int, int, np.ndarray]:
    """(bars, topk, records (n, 11)) of a fetcher-written file."""
    with open(path, "rb") as f:
        data = f.read()
    version, bars, topk = _HEAD.unpack_from(data)
    if version != 1:
        raise ValueError(f"{path}: cycle cache version {version}")
    n = (len(data) - _HEAD.size) // (8 * len(FETCHER_FIELDS))
    rec = np.frombuffer(data, dtype="<f8", count=n * len(FETCHER_FIELDS), offset=_HEAD.size)
    return bars, topk, rec.reshape(n, len(FETCHER_FIELDS)).copy()


def warmup_buffers(cycles: np.ndarray, out_len: int, stride: int, top_k: int, hop: int, fft_window: int, got: int,
                   period_seconds: int, music_only: bool = True, use_weights: bool = True, min_coherence: float = 0.05,
                   min_score: float = 0.01, min_snr_db: float = -40.0) -> np.ndarray:
    """Batch-warmup reconstruction of the per-bar buffers from cycle records
    (1.1.0:1044-1099; defaults InpMusicOnly, InpUseMusicWeights, InpMinCoherence,
    InpMinScore, InpMinSnrDb of 1.1.0:64, 73-76).  Returns (got, 20) in
    INDICATOR_FIELDS order, EMPTY_VALUE where no cycle wrote.
    """
    c = np.asarray(cycles, dtype=np.float64).reshape(-1)
    buf = np.full((got, len(INDICATOR_FIELDS)), EMPTY_VALUE)
    two_pi = 6.28318530717958647692
    for i in range(out_len):
        base = i * stride
        method_id = int(c[base + 14]) if stride > 14 else 0
        if music_only and method_id != 1:
            continue
        amp, freq, period, phase = c[base], c[base + 1], c[base + 2], c[base + 3]
        eta_sec = c[base + 5]
        energy, coher, snr, eigen, score, etac = (c[base + 6], c[base + 7], c[base + 8], c[base + 10], c[base + 11],
                                                  c[base + 13])
        w_energy, w_coher, w_score = max(energy, 0.0), max(coher, 0.0), max(score, 0.0)
        snr_eff = max(snr, min_snr_db)
        w_snr = 1.0 / (1.0 + math.pow(10.0, -snr_eff / 10.0))
        weight = (w_energy * w_coher * w_score * w_snr) if use_weights else 1.0
        if coher < min_coherence or score < min_score:
            weight = 0.0
        window_idx = i // top_k
        start_bar = window_idx * hop
        if start_bar >= got:
            continue
        omega = two_pi * freq
        span = min(fft_window - 1, got - start_bar - 1)
        slot = i % top_k
        if slot > 1:  # 1.1.0 keeps two waves: slot 0 -> buffers 1, every other slot -> buffers 2
            slot = 1
        k = np.arange(span + 1, dtype=np.float64)
        theta = phase - omega * k
        idx = start_bar + np.arange(span + 1)
        cols = np.array([0, 2, 4, 6, 8, 10, 12, 14, 16, 18]) + slot
        vals = np.stack([amp * weight * np.sin(theta), np.full_like(k, period),
                         np.maximum(eta_sec - k * period_seconds, 0.0), theta, np.full_like(k, energy),
                         np.full_like(k, coher), np.full_like(k, snr), np.full_like(k, score), np.full_like(k, eigen),
                         np.full_like(k, etac)], axis=1)
        buf[idx[:, None], cols[None, :]] = vals
    return buf


def fetcher_to_indicator(fetcher_path: str, indicator_path: str, top_k: int, hop: int, fft_window: int,
                         period_seconds: int, method: int = 1, **filters) -> np.ndarray:
    """Build-defined conversion of a fetcher cache into the indicator's layout.

    The missing record fields (eta_bars, residual_power, kalman_pred) are 0;
    the method id, absent from the fetcher file, is taken from the file
    name's ``_m<method>`` (the fetcher's InpMethod).  The records are fed to
    :func:`warmup_buffers` with the fetcher's bar count, and the result is
    written with :func:`save_cycle_cache`.
    """
    bars, _, rec = read_fetcher_cycle_cache(fetcher_path)
    full = np.zeros((rec.shape[0], len(CYCLE_RECORD)))
    full[:, FETCHER_FIELDS] = rec
    full[:, 14] = method
    buf = warmup_buffers(full, rec.shape[0], len(CYCLE_RECORD), top_k, hop, fft_window, bars, period_seconds,
                         **filters)
    save_cycle_cache(indicator_path, buf)
    return buf
