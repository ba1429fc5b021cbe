"""C5 per window length: one grouped launch over the 7 symbols of one length (wsp_group_*), timed with
HIP events on its stream for a list of segment lengths (wsp_group_set_segment; 0 = the library's policy).
Prints ms per launch and the output write rate (the slide's bound) per (N, segment).

    python scripts/c5_len_sweep.py [reps] [seg seg ...]
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "fft-wavespec_amd"))

import torch  # noqa: E402

from wavespec_amd import bridge, synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    segs = [int(x) for x in sys.argv[2:]] if len(sys.argv) > 2 else [0, 32, 64, 96, 128, 192, 256, 384, 512]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    bars = 20000
    res = []
    for n in (4096, 2048, 1024, 512):
        nwin = bars - n + 1
        series = [synth.random_walk_torch(bars, 100 + i, dev) for i in range(7)]
        outs = [torch.empty(nwin * (n // 2), dtype=torch.float64, device=dev) for _ in range(7)]
        ptrs = ([x.data_ptr() for x in series], [o.data_ptr() for o in outs])
        out_bytes = 7 * nwin * (n // 2) * 8
        for seg in segs:
            g = bridge.Group(0, [n] * 7, [nwin] * 7)
            if seg:
                g.set_segment(seg)
            for _ in range(30):
                g.execute(*ptrs, stream.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                g.execute(*ptrs, stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            g.close()
            r = {"n": n, "seg": seg, "ms": ms, "out_TBps": out_bytes / ms / 1e9}
            res.append(r)
            print(json.dumps(r), flush=True)
    best = {}
    for r in res:
        if r["n"] not in best or r["ms"] < best[r["n"]]["ms"]:
            best[r["n"]] = r
    print(json.dumps({"best": best, "sum_best_ms": sum(b["ms"] for b in best.values()),
                      "sum_auto_ms": sum(r["ms"] for r in res if r["seg"] == 0)}))


if __name__ == "__main__":
    main()
