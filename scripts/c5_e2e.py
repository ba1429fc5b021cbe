"""C5 end to end through the host API ("report end-to-end separately"): 28 symbols x 20000
bars, N = 512 / 1024 / 2048 / 4096 (7 symbols each), hop = 1, fp64 Hann, from 28 threads at once -- one
per chart, as MT5 runs them -- with the series and the spectra in host memory.  Never bench.py's `value`.

  fetcher    each thread replays WaveCyclesBatchFetcher::OnTimer (WaveCyclesBatchFetcher.mq5:104-133)
             on the spectrum batch API: gpu_submit_spectrum_batch (copies the series), then the fetcher's
             own poll loop (4000 tries, Sleep(5) only on OK with ready == 0) with
             gpu_try_get_spectrum_batch, then gpu_free_job
  registered each thread registers its series and output array once (gpu_register_host, the pinned
             FeedCache) and calls the synchronous gpu_spectrum_batch: DMA in place both ways

ctypes releases the GIL inside every library call, so the 28 threads overlap in the library as MT5's
chart threads would.  Prints one JSON object: seconds per round (best of 3), windows/s, host bytes/s.

    python scripts/c5_e2e.py [fetcher|registered]
"""
import ctypes as C
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "fft-wavespec_amd"))
from wavespec_amd import bridge, synth  # noqa: E402

MODE = sys.argv[1] if len(sys.argv) > 1 else "fetcher"
BARS, LENS = 20000, (512, 1024, 2048, 4096)
lens = [LENS[s // 7] for s in range(28)]
nwins = [BARS - n + 1 for n in lens]
series = [synth.random_walk(BARS, 100 + s) for s in range(28)]
outs = [np.empty(nw * (n // 2)) for n, nw in zip(lens, nwins)]
lib = bridge.lib()


def fetcher(s, res):
    jid = C.c_int64(0)
    st = lib.gpu_submit_spectrum_batch(bridge._dptr(series[s]), BARS, lens[s], 1, 0, 1, 0, 0, 0, C.byref(jid))
    if st != 0 or jid.value == 0:
        res[s] = ("submit", st)
        return
    ready, got = C.c_int32(0), C.c_int32(0)
    tries = 0
    while tries < 4000 and ready.value == 0:  # WaveCyclesBatchFetcher.mq5:127-131
        st = lib.gpu_try_get_spectrum_batch(jid.value, bridge._dptr(outs[s]), outs[s].size, C.byref(got), C.byref(ready))
        if st == 0 and ready.value == 0:
            time.sleep(0.005)
        elif st != 0 and st != bridge.NOT_READY:
            break
        tries += 1
    lib.gpu_free_job(jid.value)
    res[s] = ("ok" if st == 0 and ready.value == 1 and got.value == nwins[s] else "fail", st, tries)


def registered(s, res):
    got = C.c_int32(0)
    st = lib.gpu_spectrum_batch(bridge._dptr(series[s]), BARS, lens[s], 1, 0, 1, 0, 0, 0, bridge._dptr(outs[s]),
                                outs[s].size, C.byref(got))
    res[s] = ("ok" if st == 0 and got.value == nwins[s] else "fail", st)


def one_round(fn):
    res = {}
    th = [threading.Thread(target=fn, args=(s, res)) for s in range(28)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    bad = {s: r for s, r in res.items() if r[0] != "ok"}
    if bad or len(res) != 28:
        raise SystemExit(f"failed symbols: {bad}")
    return dt, res


bridge.init(0, 64)
try:
    if MODE == "registered":
        t0 = time.perf_counter()
        for a in series + outs:
            bridge.register_host(a)
        t_reg = time.perf_counter() - t0
    fn = registered if MODE == "registered" else fetcher
    one_round(fn)  # warm: code objects, tables, staging pools
    times, polls = [], []
    for _ in range(3):
        dt, res = one_round(fn)
        times.append(dt)
        if MODE == "fetcher":
            polls.append(max(r[2] for r in res.values()))
    if MODE == "registered":
        for a in series + outs:
            bridge.unregister_host(a)
finally:
    bridge.shutdown()
best = min(times)
out_bytes = sum(o.size for o in outs) * 8
in_bytes = 28 * BARS * 8
print(json.dumps({
    "config": "c5: 28 symbols x 20000 bars, N in (512, 1024, 2048, 4096), hop 1, f64 Hann, |X|^2", "mode": MODE,
    "threads": 28, "seconds": times, "windows_per_s": sum(nwins) / best, "host_bytes_per_s": (out_bytes + in_bytes) / best,
    "output_bytes": out_bytes, "max_polls": polls or None,
    "register_seconds": t_reg if MODE == "registered" else None,
    "note": "host memory both ways through the C ABI from 28 threads, 1 GPU; fetcher mode sleeps 5 ms per pending poll "
            "as WaveCyclesBatchFetcher.mq5:130 does"}))
