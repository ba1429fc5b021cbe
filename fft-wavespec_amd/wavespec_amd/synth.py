"""Synthetic price series for the BASELINE configurations.

There is no market data in this environment; every config runs on seeded
synthetic bars of the shape the reference consumes (close prices ~1.1).
"""
from __future__ import annotations

import numpy as np


def sine_noise_window(n: int = 1024, seed: int = 1234) -> np.ndarray:
    """C1: x[t] = 1.1 + 0.002 sin(2 pi t/50) + 0.001 sin(2 pi t/23 + 0.3) + 5e-4 N(0,1)."""
    t = np.arange(n, dtype=np.float64)
    rng = np.random.default_rng(seed)
    return (1.1 + 0.002 * np.sin(2 * np.pi * t / 50) + 0.001 * np.sin(2 * np.pi * t / 23 + 0.3)
            + 5e-4 * rng.standard_normal(n))


def random_walk(length: int, seed: int, step: float = 1e-4) -> np.ndarray:
    """C2..C5: 1.1 + cumsum(step * N(0,1)) + 0.002 sin(2 pi t/50)."""
    rng = np.random.default_rng(seed)
    t = np.arange(length, dtype=np.float64)
    return 1.1 + np.cumsum(step * rng.standard_normal(length)) + 0.002 * np.sin(2 * np.pi * t / 50)


def random_walk_torch(length: int, seed: int, device, dtype=None, step: float = 1e-4):
    """Same generator shape built directly in HBM (bench: inputs resident on device)."""
    import torch
    dtype = dtype or torch.float64
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    noise = torch.randn(length, generator=g, device=device, dtype=torch.float64)
    t = torch.arange(length, device=device, dtype=torch.float64)
    x = 1.1 + torch.cumsum(step * noise, 0) + 0.002 * torch.sin(2 * np.pi * t / 50)
    return x.to(dtype)


# (name, windows, N, hop, precision, detrend, window, seed)  -- BASELINE.json configs
CONFIGS = {
    "c1": dict(windows=1, n=1024, hop=1024, precision="f64", detrend="none", window="hann", seed=1234),
    "c2": dict(windows=4096, n=1024, hop=1024, precision="f64", detrend="none", window="hann", seed=7),
    "c3": dict(windows=65536, n=4096, hop=4096, precision="f32", detrend="kalman", window="hann", seed=11),
    "north_star": dict(windows=65536, n=4096, hop=4096, precision="f64", detrend="none", window="hann", seed=11),
    "c4": dict(windows=1048576, n=2048, hop=1, precision="f64", detrend="none", window="hann", seed=13),
    # SURVEY 8f rows on the north-star shape (not the headline metric): fused consumers of the
    # spectrum and the inverse transform
    "ns_topk": dict(windows=65536, n=4096, hop=4096, precision="f64", detrend="none", window="hann", seed=11,
                    output="topk"),
    # C4's batch reduced on device to the reference's top-8 scan (SURVEY 8f rank 1 on the hop = 1 shape)
    "c4_topk": dict(windows=1048576, n=2048, hop=1, precision="f64", detrend="none", window="hann", seed=13,
                    output="topk"),
    "ns_phase": dict(windows=65536, n=4096, hop=4096, precision="f64", detrend="none", window="hann", seed=11,
                     output="phase"),
    "ns_topk_phase": dict(windows=65536, n=4096, hop=4096, precision="f64", detrend="none", window="hann",
                          seed=11, output="topk_phase"),
    "inverse": dict(windows=65536, n=4096, hop=4096, precision="f64", detrend="none", window="none", seed=11,
                    output="inverse"),
    # the legacy default InpFFTWindow = 65536 (four-step path), north-star bytes
    "large": dict(windows=4096, n=65536, hop=65536, precision="f64", detrend="none", window="hann", seed=11),
    "large_131072": dict(windows=2048, n=131072, hop=131072, precision="f64", detrend="none", window="hann", seed=11),
    "large_262144": dict(windows=1024, n=262144, hop=262144, precision="f64", detrend="none", window="hann", seed=11),
}


def series_len(cfg: dict) -> int:
    return (cfg["windows"] - 1) * cfg["hop"] + cfg["n"]
