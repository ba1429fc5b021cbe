"""ctypes binding of libmtbridge.so (include/mtbridge.h).

This is the Python view of the C ABI that replaces ``mt-bridge.dll``
(reference ``Include/imports.mqh:4-20``).  It adds nothing to the compute
path: every call goes straight into the HIP library.  If the library is
missing the import of :func:`lib` raises -- there is no CPU fallback
(reference ``CHANGELOG.md:5,15``: "sem fallback CPU").
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_ROOT = Path(__file__).resolve().parent.parent  # fft-wavespec_amd/
LIB_PATH = PKG_ROOT / "lib" / "libmtbridge.so"

# status codes (L/WaveSpecZZ_gpu_wip.mq5:263-269)
OK, BAD_ARGS, BACKEND_UNAVAILABLE, TIMEOUT, INTERNAL_ERROR, NOT_READY, NO_MEM = 0, -1, -2, -3, -4, -5, -6
STATUS_NAMES = {OK: "OK", BAD_ARGS: "BAD_ARGS", BACKEND_UNAVAILABLE: "BACKEND_UNAVAILABLE", TIMEOUT: "TIMEOUT",
                INTERNAL_ERROR: "INTERNAL", NOT_READY: "NOT_READY", NO_MEM: "NO_MEM"}
DETREND = {"none": 0, "mean": 1, "iir": 2, "kalman": 3}
WINDOW = {"none": 0, "hann": 1, "hamming": 2, "blackman": 3, "bartlett": 4}
PRECISION = {"f64": 0, "f32": 1}
OUTPUT = {"power": 0, "packed": 1, "topk": 2, "phase": 3, "topk_phase": 4}
PHASE_METHOD = {"unwrapped": 0, "wrapped": 1, "group_delay": 2}

_d = C.POINTER(C.c_double)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)

# name -> (restype, argtypes); exactly the prototypes of include/mtbridge.h
SIGNATURES = {
    "gpu_init": (C.c_int32, [C.c_int32, C.c_int32]),
    "gpu_shutdown": (None, []),
    "gpu_fft_real_forward": (C.c_int32, [_d, C.c_int32, _d]),
    "gpu_extract_cycles": (C.c_int32, [_d, C.c_int32, C.c_int32, C.c_double, C.c_double, C.c_double, C.c_int32,
                                       C.c_int32, _d, C.c_int32, C.c_int32, _i32p]),
    "gpu_submit_extract_cycles": (C.c_int32, [_d, C.c_int32, C.c_int32, C.c_double, C.c_double, C.c_double,
                                              C.c_int32, C.c_int32, _i64p]),
    "gpu_try_get_cycles": (C.c_int32, [C.c_int64, _d, C.c_int32, C.c_int32, _i32p, _i32p]),
    "gpu_submit_extract_cycles_batch": (C.c_int32, [_d, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_double,
                                                    C.c_double, C.c_double, C.c_int32, C.c_int32, C.c_int32, _i64p]),
    "gpu_try_get_cycles_batch": (C.c_int32, [C.c_int64, _d, C.c_int32, _i32p, _i32p]),
    "gpu_free_job": (C.c_int32, [C.c_int64]),
    "gpu_get_last_error_w": (C.c_int32, [C.POINTER(C.c_uint16), C.c_int32]),
    "gpu_fft_real_forward_batch": (C.c_int32, [_d, C.c_int32, C.c_int32, _d]),
    "gpu_fft_real_inverse": (C.c_int32, [_d, C.c_int32, _d]),
    "gpu_fft_real_inverse_batch": (C.c_int32, [_d, C.c_int32, C.c_int32, _d]),
    "gpu_spectral_phase_unwrap": (C.c_int32, [_d, C.c_int32, C.c_int32, _d, C.c_int32]),
    "gpu_spectrum_topk_phase_batch": (C.c_int32, [_d, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                                  C.c_int32, C.c_int32, C.c_double, C.c_double, _d, C.c_int32,
                                                  _i32p]),
    "gpu_spectrum_batch": (C.c_int32, [_d, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                       C.c_int32, C.c_int32, _d, C.c_int32, _i32p]),
    "gpu_submit_spectrum_batch": (C.c_int32, [_d, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                              C.c_int32, C.c_int32, C.c_int32, _i64p]),
    "gpu_try_get_spectrum_batch": (C.c_int32, [C.c_int64, _d, C.c_int32, _i32p, _i32p]),
    "gpu_set_kalman_params": (C.c_int32, [_d, C.c_int32]),
    "gpu_register_host": (C.c_int32, [_d, C.c_int64]),
    "gpu_unregister_host": (C.c_int32, [_d]),
    "gpu_set_host_locking": (C.c_int32, [C.c_int32]),
    "gpu_session_id": (C.c_int64, []),
    "gpu_spectrum_topk_batch": (C.c_int32, [_d, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                            C.c_int32, C.c_int32, C.c_double, C.c_double, _d, C.c_int32, _i32p]),
    "wsp_plan_set_topk": (C.c_int32, [C.c_int64, C.c_int32, C.c_double, C.c_double]),
    "wsp_plan_set_algorithm": (C.c_int32, [C.c_int64, C.c_int32]),
    "wsp_plan_get_algorithm": (C.c_int32, [C.c_int64]),
    "wsp_plan_set_slide_segment": (C.c_int32, [C.c_int64, C.c_int64]),
    "wsp_plan_set_seed_chain": (C.c_int32, [C.c_int64, C.c_int32]),
    "wsp_plan_set_trace": (C.c_int32, [C.c_int64, C.c_void_p, C.c_int64]),
    "wsp_plan_set_variant": (C.c_int32, [C.c_int64, C.c_int32]),
    "wsp_plan_set_scan_flags": (C.c_int32, [C.c_int64, C.c_void_p]),
    "wsp_plan_set_chunk": (C.c_int32, [C.c_int64, C.c_int64]),
    "wsp_plan_set_grid": (C.c_int32, [C.c_int64, C.c_int32]),
    "wsp_plan_create": (C.c_int64, [C.c_int32, C.c_int32, C.c_int64, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                    C.c_int32, C.c_int32]),
    "wsp_plan_create_inverse": (C.c_int64, [C.c_int32, C.c_int32, C.c_int64]),
    "wsp_plan_execute": (C.c_int32, [C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]),
    "wsp_plan_algorithmic_bytes": (C.c_int64, [C.c_int64]),
    "wsp_plan_destroy": (C.c_int32, [C.c_int64]),
    "wsp_group_create": (C.c_int64, [C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.c_int32,
                                     C.c_int32, C.c_int32]),
    "wsp_group_execute": (C.c_int32, [C.c_int64, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_void_p]),
    "wsp_group_algorithmic_bytes": (C.c_int64, [C.c_int64]),
    "wsp_group_launches": (C.c_int32, [C.c_int64]),
    "wsp_group_set_streams": (C.c_int32, [C.c_int64, C.c_int32]),
    "wsp_group_set_segment": (C.c_int32, [C.c_int64, C.c_int64]),
    "wsp_group_set_mode": (C.c_int32, [C.c_int64, C.c_int32]),
    "wsp_group_destroy": (C.c_int32, [C.c_int64]),
    "wsp_group_set_trace": (C.c_int32, [C.c_int64, C.c_void_p, C.c_int64]),
    "wsp_group_last_tasks": (C.c_int64, [C.c_int64]),
    "wsp_version": (C.c_char_p, []),
}

_LIB = None


class BridgeError(RuntimeError):
    def __init__(self, fn: str, status: int, reason: str):
        super().__init__(f"{fn} -> {STATUS_NAMES.get(status, status)}: {reason}")
        self.status = status
        self.reason = reason


def lib() -> C.CDLL:
    """Load libmtbridge.so (fails loudly when it has not been built)."""
    global _LIB
    if _LIB is None:
        path = Path(os.environ.get("WSP_MTBRIDGE_LIB", LIB_PATH))
        if not path.exists():
            raise FileNotFoundError(f"{path} not built: run __graft_entry__.build() or `make -C fft-wavespec_amd`")
        h = C.CDLL(str(path))
        for name, (res, args) in SIGNATURES.items():
            f = getattr(h, name)
            f.restype = res
            f.argtypes = args
        _LIB = h
    return _LIB


def last_error() -> str:
    """gpu_get_last_error_w as MQL reads it: ShortArrayToString(buf, 0, n-1)."""
    buf = (C.c_uint16 * 256)()
    n = lib().gpu_get_last_error_w(buf, 256)
    return "".join(chr(buf[i]) for i in range(n - 1)) if n > 0 else "n/a"


def _check(fn: str, st: int) -> int:
    if st != OK:
        raise BridgeError(fn, st, last_error())
    return st


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(_d)


def init(device_index: int = 0, stream_count: int = 64) -> None:
    _check("gpu_init", lib().gpu_init(device_index, stream_count))


def shutdown() -> None:
    lib().gpu_shutdown()


def fft_real_forward(x: np.ndarray) -> np.ndarray:
    """gpu_fft_real_forward: packed out[2k]=Re X_k, out[2k+1]=Im X_k, k < N/2."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    _check("gpu_fft_real_forward", lib().gpu_fft_real_forward(_dptr(x), x.size, _dptr(out)))
    return out


def fft_real_forward_batch(windows: np.ndarray) -> np.ndarray:
    w = np.ascontiguousarray(windows, dtype=np.float64)
    out = np.empty_like(w)
    _check("gpu_fft_real_forward_batch",
           lib().gpu_fft_real_forward_batch(_dptr(w), w.shape[1], w.shape[0], _dptr(out)))
    return out


def fft_real_inverse(spec: np.ndarray) -> np.ndarray:
    """gpu_fft_real_inverse: packed spectrum (gpu_fft_real_forward layout) -> samples."""
    spec = np.ascontiguousarray(spec, dtype=np.float64)
    out = np.empty_like(spec)
    _check("gpu_fft_real_inverse", lib().gpu_fft_real_inverse(_dptr(spec), spec.size, _dptr(out)))
    return out


def fft_real_inverse_batch(spectra: np.ndarray) -> np.ndarray:
    s = np.ascontiguousarray(spectra, dtype=np.float64)
    out = np.empty_like(s)
    _check("gpu_fft_real_inverse_batch",
           lib().gpu_fft_real_inverse_batch(_dptr(s), s.shape[1], s.shape[0], _dptr(out)))
    return out


def spectral_phase_unwrap(spec: np.ndarray, method="unwrapped") -> np.ndarray:
    """gpu_spectral_phase_unwrap over a packed spectrum -> spectrum_len/2 values."""
    spec = np.ascontiguousarray(spec, dtype=np.float64)
    out = np.empty(spec.size // 2)
    _check("gpu_spectral_phase_unwrap",
           lib().gpu_spectral_phase_unwrap(_dptr(spec), spec.size, PHASE_METHOD[method], _dptr(out), out.size))
    return out


def _record(window_len: int, output: str, top_k: int = 8) -> int:
    return {"packed": window_len, "topk": 4 * top_k, "topk_phase": 6 * top_k,
            "phase": 3 * (window_len // 2)}.get(output, window_len // 2)


def spectrum_batch(series: np.ndarray, window_len: int, hop: int, detrend="none", window="hann",
                   trend_period: int = 0, precision="f64", output="power", max_records: int | None = None,
                   out: np.ndarray | None = None) -> np.ndarray:
    """gpu_spectrum_batch over a chronological series -> (nwin, record) array.  `out`: a
    caller-owned C-contiguous float64 array of at least nwin * record elements (the library
    drains its pinned output ring into it)."""
    s = np.ascontiguousarray(series, dtype=np.float64)
    nwin = 1 + (s.size - window_len) // hop
    rec = _record(window_len, output)
    if max_records is not None:
        nwin = min(nwin, max_records)
    if out is None:
        out = np.empty((nwin, rec), dtype=np.float64)
    elif out.dtype != np.float64 or not out.flags.c_contiguous or out.size < nwin * rec:
        raise ValueError("out must be a C-contiguous float64 array of >= nwin * record elements")
    else:
        out = out.reshape(-1)[: nwin * rec].reshape(nwin, rec)
    n_out = C.c_int32(0)
    _check("gpu_spectrum_batch",
           lib().gpu_spectrum_batch(_dptr(s), s.size, window_len, hop, DETREND[detrend], WINDOW[window],
                                    trend_period, PRECISION[precision], OUTPUT[output], _dptr(out), out.size,
                                    C.byref(n_out)))
    return out[: n_out.value]


def spectrum_topk_batch(series: np.ndarray, window_len: int, hop: int, detrend="none", window="hann",
                        trend_period: int = 0, precision="f64", top_k: int = 8, min_period: float = 18.0,
                        max_period: float = 200.0) -> np.ndarray:
    """gpu_spectrum_topk_batch -> (nwin, top_k, 4) records [bin, power, Re X, Im X]."""
    s = np.ascontiguousarray(series, dtype=np.float64)
    nwin = 1 + (s.size - window_len) // hop
    out = np.empty((nwin, top_k, 4), dtype=np.float64)
    n_out = C.c_int32(0)
    _check("gpu_spectrum_topk_batch",
           lib().gpu_spectrum_topk_batch(_dptr(s), s.size, window_len, hop, DETREND[detrend], WINDOW[window],
                                         trend_period, PRECISION[precision], top_k, min_period, max_period,
                                         _dptr(out), out.size, C.byref(n_out)))
    return out[: n_out.value]


def spectrum_topk_phase_batch(series: np.ndarray, window_len: int, hop: int, detrend="none", window="hann",
                              trend_period: int = 0, top_k: int = 8, min_period: float = 18.0,
                              max_period: float = 200.0) -> np.ndarray:
    """gpu_spectrum_topk_phase_batch -> (nwin, top_k, 6) [bin, power, Re, Im, phase, group delay]."""
    s = np.ascontiguousarray(series, dtype=np.float64)
    nwin = 1 + (s.size - window_len) // hop
    out = np.empty((nwin, top_k, 6), dtype=np.float64)
    n_out = C.c_int32(0)
    _check("gpu_spectrum_topk_phase_batch",
           lib().gpu_spectrum_topk_phase_batch(_dptr(s), s.size, window_len, hop, DETREND[detrend], WINDOW[window],
                                               trend_period, top_k, min_period, max_period, _dptr(out), out.size,
                                               C.byref(n_out)))
    return out[: n_out.value]


def submit_spectrum_batch(series: np.ndarray, window_len: int, hop: int, detrend="none", window="hann",
                          trend_period: int = 0, precision="f64", output="power") -> int:
    s = np.ascontiguousarray(series, dtype=np.float64)
    jid = C.c_int64(0)
    _check("gpu_submit_spectrum_batch",
           lib().gpu_submit_spectrum_batch(_dptr(s), s.size, window_len, hop, DETREND[detrend], WINDOW[window],
                                           trend_period, PRECISION[precision], OUTPUT[output], C.byref(jid)))
    return jid.value


def try_get_spectrum_batch(job_id: int, out: np.ndarray):
    """Returns (status, ready, out_len) exactly as the ABI reports them."""
    n = C.c_int32(0)
    ready = C.c_int32(0)
    st = lib().gpu_try_get_spectrum_batch(job_id, _dptr(out), out.size, C.byref(n), C.byref(ready))
    return st, ready.value, n.value


def free_job(job_id: int) -> int:
    return lib().gpu_free_job(job_id)


def register_host(a: np.ndarray) -> None:
    """gpu_register_host: record a C-contiguous float64 array (FeedCache history, output arrays) for the
    session.  Round 6: nothing is page-locked -- calls stage through the library's own pinned buffers
    (DESIGN.md 4.2); overlapping registrations are refused."""
    if a.dtype != np.float64 or not a.flags.c_contiguous:
        raise ValueError("register_host needs a C-contiguous float64 array")
    _check("gpu_register_host", lib().gpu_register_host(_dptr(a), a.size))


def unregister_host(a: np.ndarray) -> None:
    """gpu_unregister_host: raises on every failure (an unknown buffer: BAD_ARGS; no session:
    BACKEND_UNAVAILABLE)."""
    _check("gpu_unregister_host", lib().gpu_unregister_host(_dptr(a)))


def set_host_locking(mode: int) -> int:
    """gpu_set_host_locking: 0 (record the range, calls stage) is the only mode and returns 0; 1 (page-lock
    caller memory, opt-in in round 5) was withdrawn in round 6 and raises BAD_ARGS."""
    r = int(lib().gpu_set_host_locking(mode))
    if r < 0:
        _check("gpu_set_host_locking", r)
    return r


def session_id() -> int:
    """gpu_session_id: > 0 for the open session (changes when a new session is opened), 0 without one."""
    return int(lib().gpu_session_id())


def set_kalman_params(params) -> None:
    p = np.ascontiguousarray(params, dtype=np.float64)
    _check("gpu_set_kalman_params", lib().gpu_set_kalman_params(_dptr(p), p.size))


class Plan:
    """Device-resident plan (wsp_plan_*): the hot path on buffers already in HBM."""

    def __init__(self, device: int, window_len: int, hop: int, n_windows: int, detrend="none", window="hann",
                 trend_period: int = 0, precision="f64", output="power"):
        self.handle = lib().wsp_plan_create(device, window_len, hop, n_windows, DETREND[detrend], WINDOW[window],
                                            trend_period, PRECISION[precision], OUTPUT[output])
        if self.handle == 0:
            raise BridgeError("wsp_plan_create", INTERNAL_ERROR, last_error())
        self.window_len, self.hop, self.n_windows = window_len, hop, n_windows
        self.output = output
        self.record = _record(window_len, output)
        self.series_len = (n_windows - 1) * hop + window_len

    @classmethod
    def inverse(cls, device: int, window_len: int, n_windows: int) -> "Plan":
        """wsp_plan_create_inverse: rows of packed spectra -> rows of samples."""
        self = cls.__new__(cls)
        self.handle = lib().wsp_plan_create_inverse(device, window_len, n_windows)
        if self.handle == 0:
            raise BridgeError("wsp_plan_create_inverse", INTERNAL_ERROR, last_error())
        self.window_len, self.hop, self.n_windows = window_len, window_len, n_windows
        self.output = "inverse"
        self.record = window_len
        self.series_len = n_windows * window_len
        return self

    def set_topk(self, top_k: int, min_period: float, max_period: float) -> None:
        _check("wsp_plan_set_topk", lib().wsp_plan_set_topk(self.handle, top_k, min_period, max_period))
        self.record = (6 if self.output == "topk_phase" else 4) * top_k

    ALGOS = {"auto": 0, "fft": 1, "slide": 2}

    def set_algorithm(self, algo: str) -> None:
        """wsp_plan_set_algorithm: "auto", "fft" or "slide" (hop = 1 seeded sliding DFT)."""
        _check("wsp_plan_set_algorithm", lib().wsp_plan_set_algorithm(self.handle, self.ALGOS[algo]))

    def set_slide_segment(self, windows: int) -> None:
        """Tuning: windows per sliding-DFT workgroup (0 = the library's policy)."""
        _check("wsp_plan_set_slide_segment", lib().wsp_plan_set_slide_segment(self.handle, windows))

    def set_seed_chain(self, segments: int) -> None:
        """Tuning: top-k segments per seed workgroup (1 = one FFT seed each, 0 = the library's policy)."""
        _check("wsp_plan_set_seed_chain", lib().wsp_plan_set_seed_chain(self.handle, segments))

    def set_trace(self, d_trace: int, capacity: int) -> None:
        """Diagnostic: timeline of the hop = 1 slide / top-k kernels or the fused large-N kernel into a device buffer
        of `capacity` int64 (include/mtbridge.h wsp_plan_set_trace)."""
        _check("wsp_plan_set_trace", lib().wsp_plan_set_trace(self.handle, d_trace, capacity))

    def set_variant(self, variant: int) -> None:
        """Ablation: the kernel form (include/mtbridge.h wsp_plan_set_variant; 0 = the library's choice)."""
        _check("wsp_plan_set_variant", lib().wsp_plan_set_variant(self.handle, variant))

    def set_chunk(self, windows: int) -> None:
        """Tuning: windows per chunk of the two-pass large-N path (0 = the library's ~192 MiB of column results)."""
        _check("wsp_plan_set_chunk", lib().wsp_plan_set_chunk(self.handle, windows))

    def set_grid(self, workgroups: int) -> None:
        """Tuning: workgroups of the FFT-kernel / inverse launch (0 = the library's 32768)."""
        _check("wsp_plan_set_grid", lib().wsp_plan_set_grid(self.handle, workgroups))

    def set_scan_flags(self, d_flags: int) -> None:
        """Diagnostics: device buffer of n_windows bytes receiving each window's top-k scan path
        (0 candidate list, 1 segment start, 2 candidate overflow), or 0 = off."""
        _check("wsp_plan_set_scan_flags", lib().wsp_plan_set_scan_flags(self.handle, C.c_void_p(d_flags)))

    def algorithm(self) -> str:
        """What the next execute runs: "fft" or "slide"."""
        return {1: "fft", 2: "slide"}[lib().wsp_plan_get_algorithm(self.handle)]

    @property
    def algorithmic_bytes(self) -> int:
        return int(lib().wsp_plan_algorithmic_bytes(self.handle))

    def execute(self, d_series: int, d_out: int, stream: int = 0) -> None:
        _check("wsp_plan_execute", lib().wsp_plan_execute(self.handle, C.c_void_p(d_series), C.c_void_p(d_out),
                                                          C.c_void_p(stream)))

    def close(self) -> None:
        if self.handle:
            lib().wsp_plan_destroy(self.handle)
            self.handle = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Group:
    """Grouped hop = 1 device plan (wsp_group_*): one series per symbol, every window of each
    (the WaveCyclesBatchFetcher shape); the members of a window length run in one launch."""

    def __init__(self, device: int, window_lens, n_windows, detrend="none", window="hann", precision="f64"):
        lens = (C.c_int32 * len(window_lens))(*window_lens)
        nws = (C.c_int64 * len(n_windows))(*n_windows)
        if len(window_lens) != len(n_windows):
            raise ValueError("one window length and one window count per member")
        self.handle = lib().wsp_group_create(device, len(window_lens), lens, nws, DETREND[detrend], WINDOW[window],
                                             PRECISION[precision])
        if self.handle == 0:
            raise BridgeError("wsp_group_create", BAD_ARGS, last_error())
        self.window_lens, self.n_windows = list(window_lens), list(n_windows)

    @property
    def algorithmic_bytes(self) -> int:
        return int(lib().wsp_group_algorithmic_bytes(self.handle))

    @property
    def launches(self) -> int:
        return int(lib().wsp_group_launches(self.handle))

    def set_streams(self, n: int) -> None:
        """Tuning: fork each execute over n internal streams (1 = the caller's stream only)."""
        _check("wsp_group_set_streams", lib().wsp_group_set_streams(self.handle, n))

    def set_segment(self, windows: int) -> None:
        """Tuning: windows per sliding-DFT workgroup (0 = the launcher's policy)."""
        _check("wsp_group_set_segment", lib().wsp_group_set_segment(self.handle, windows))

    MODES = {"auto": 0, "per-length": 1, "mixed-b4": 2, "mixed-tail-half": 3, "mixed-uniform": 4, "mixed-lds-seeds": 5,
             "mixed-plain-stores": 6}

    def set_mode(self, mode: str) -> None:
        """"auto": one mixed-length persistent launch where eligible; "per-length": one launch per window length;
        "mixed-b4" / "mixed-tail-half" / "mixed-uniform": ablations of the mixed launch (four bins per thread for
        N <= 1024 / half-length segments for the shortest window length at every batch size / never) --
        wsp_group_set_mode 0..4, include/mtbridge.h."""
        _check("wsp_group_set_mode", lib().wsp_group_set_mode(self.handle, self.MODES[mode]))

    def set_trace(self, d_trace: int, capacity_tasks: int) -> None:
        """Diagnostic: per-task timeline of the mixed launch into a device buffer of 4 x capacity int64."""
        _check("wsp_group_set_trace", lib().wsp_group_set_trace(self.handle, C.c_void_p(d_trace), capacity_tasks))

    @property
    def last_tasks(self) -> int:
        return int(lib().wsp_group_last_tasks(self.handle))

    def execute(self, d_series, d_out, stream: int = 0) -> None:
        """d_series / d_out: device pointers (ints), one per member."""
        n = len(self.window_lens)
        if len(d_series) != n or len(d_out) != n:
            raise ValueError(f"{n} members: one series and one output pointer each")
        ins = (C.c_void_p * n)(*d_series)
        outs = (C.c_void_p * n)(*d_out)
        _check("wsp_group_execute", lib().wsp_group_execute(self.handle, ins, outs, C.c_void_p(stream)))

    def close(self) -> None:
        if self.handle:
            lib().wsp_group_destroy(self.handle)
            self.handle = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
