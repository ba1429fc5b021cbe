"""C5 per window length: one grouped launch over the 7 symbols of one length (wsp_group_*), timed with
HIP events on its stream for a list of segment lengths (wsp_group_set_segment; 0 = the library's policy).
Prints ms per launch and the output write rate (the slide's bound) per (N, segment).

    python scripts/c5_len_sweep.py [reps] [seg seg ...] [--mode auto|per-length|mixed-b4|mixed-nt] [--lens 4096,512]

(round 4: a one-length group runs the mixed persistent launch by default, `--mode per-length` the round-3 one)
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "fft-wavespec_amd"))

import torch  # noqa: E402

from wavespec_amd import bridge, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("reps", nargs="?", type=int, default=50)
    ap.add_argument("segs", nargs="*", type=int)
    ap.add_argument("--mode", default="auto")
    ap.add_argument("--lens", default="4096,2048,1024,512")
    args = ap.parse_args()
    reps = args.reps
    segs = args.segs or [0, 32, 64, 96, 128, 192, 256, 384, 512]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    bars = 20000
    res = []
    for n in [int(x) for x in args.lens.split(",")]:
        nwin = bars - n + 1
        series = [synth.random_walk_torch(bars, 100 + i, dev) for i in range(7)]
        outs = [torch.empty(nwin * (n // 2), dtype=torch.float64, device=dev) for _ in range(7)]
        ptrs = ([x.data_ptr() for x in series], [o.data_ptr() for o in outs])
        out_bytes = 7 * nwin * (n // 2) * 8
        for seg in segs:
            g = bridge.Group(0, [n] * 7, [nwin] * 7)
            g.set_mode(args.mode)
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
            r = {"n": n, "seg": seg, "mode": args.mode, "ms": ms, "out_TBps": out_bytes / ms / 1e9}
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
