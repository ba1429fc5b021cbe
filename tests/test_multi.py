"""Multi-rank paths on CPU with gloo (world_size 2): bench.py's barrier /
max-over-ranks timing, and window sharding with halos reproducing the
single-process spectra (the exchange-free decomposition of SURVEY 8e)."""
import os
import socket
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT
from wavespec_amd import sharding, synth


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))


def _bench_worker(rank, world, port, q):
    _env(rank, world, port)
    import sys
    sys.path.insert(0, str(ROOT))
    import bench
    ctl = bench.Control(world)
    secs = bench.timed_steps(lambda: time.sleep(0.02 * (rank + 1)), lambda: None, ctl, steps=5, warmup=1)
    total = ctl.sum(float(100 * (rank + 1)))
    q.put((rank, secs, total))
    ctl.close()


def test_bench_control_gloo_world2():
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, s0, t0), (_, s1, t1) = res
    assert s0 == s1 and s0 >= 5 * 0.04 * 0.95  # max over ranks = the slow rank's time
    assert t0 == t1 == 300.0


def _shard_worker(rank, world, port, q):
    _env(rank, world, port)
    import sys
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    n, hop, W = 256, 37, 41
    s = synth.random_walk((W - 1) * hop + n, seed=5)
    w0, nw = sharding.shard_windows(W, world, rank)
    a, b = sharding.shard_series_slice(w0, nw, hop, n)
    local = oracle.batch_spectrum(s[a:b], n, hop, "iir", "hann", 64)
    assert local.shape[0] == nw
    per = -(-W // world)
    buf = torch.zeros(per, n // 2, dtype=torch.float64)
    buf[:nw] = torch.from_numpy(local)
    out = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(out, buf)  # test-only gather: the product path never exchanges
    full = torch.cat(out)[:W].numpy()
    q.put((rank, float(np.max(np.abs(full - oracle.batch_spectrum(s, n, hop, "iir", "hann", 64))))))
    dist.destroy_process_group()


def test_window_shards_with_halo_gloo_world2():
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(err == 0.0 for _, err in res)


@pytest.mark.parametrize("W,G", [(65536, 8), (10, 3), (3, 8), (1, 1)])
def test_shard_cover(W, G):
    seen = []
    for g in range(G):
        w0, nw = sharding.shard_windows(W, G, g)
        seen.extend(range(w0, w0 + nw))
    assert seen == list(range(W))


def _bench_line(*args, env=None):
    import json
    import subprocess
    import sys
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True, timeout=300,
                       env=env)
    return r, [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_gpus2_spawns_ranks_and_shards_c4():
    """`bench.py --gpus 2` outside torchrun starts 2 ranks (gloo rendezvous on 127.0.0.1) that split C4's
    1,048,576 hop=1 windows into contiguous ranges, each reading its slice plus the N - hop halo."""
    r, lines = _bench_line("--gpus", "2", "--config", "c4", "--scaling", "strong", "--plan-only")
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = lines
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    s0, s1 = line["shards"]
    n, hop, W = 2048, 1, 1048576
    assert s0["w0"] == 0 and s1["w0"] == s0["windows"] and s0["windows"] + s1["windows"] == W
    for sh in (s0, s1):
        a, b = sh["series"]
        assert a == sh["w0"] * hop and b == (sh["w0"] + sh["windows"] - 1) * hop + n
    assert s0["series"][1] - s1["series"][0] == n - hop  # the halo both ranks read


def test_bench_c5_strong_symbols_partition():
    r, lines = _bench_line("--gpus", "2", "--config", "c5", "--scaling", "strong", "--c5-shard", "symbols",
                           "--plan-only")
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = lines
    syms = sorted(s for sh in line["shards"] for s in sh["symbols"])
    assert syms == list(range(28))
    assert sum(sh["windows"] for sh in line["shards"]) == 506268
    lens = (512, 1024, 2048, 4096)
    out_bytes = [sum((20000 - lens[s // 7] + 1) * lens[s // 7] // 2 for s in sh["symbols"]) for sh in line["shards"]]
    assert max(out_bytes) / min(out_bytes) < 1.05  # balanced by the bytes each rank writes


@pytest.mark.parametrize("split", ["split", "split-time"])
def test_bench_c5_strong_split_pieces(split):
    """C5 cut on one cost line (McNaughton wrap-around, sharding.split_symbols) over a real 2-rank gloo
    rendezvous, and over 8 ranks through --emulate-shard R/8 (one rank's plan on one process): the pieces
    cover every window of every symbol exactly once, each rank's cost is within one window of the mean, and
    no symbol is cut more than G - 1 times."""
    import bench
    lens = (512, 1024, 2048, 4096)
    nw = [20000 - lens[s // 7] + 1 for s in range(28)]
    cost = [(n // 2 if split == "split" else bench.C5_TIME_WEIGHTS[n]) for n in (lens[s // 7] for s in range(28))]
    r, lines = _bench_line("--gpus", "2", "--config", "c5", "--scaling", "strong", "--c5-shard", split, "--plan-only")
    assert r.returncode == 0, r.stderr[-2000:]
    two = lines[0]["shards"]
    for g, shards in ((2, two), (8, None)):
        if shards is None:
            shards = []
            for rk in range(8):
                r, ln = _bench_line("--config", "c5", "--emulate-shard", f"{rk}/8", "--c5-shard", split, "--plan-only")
                assert r.returncode == 0, r.stderr[-2000:]
                shards += ln[0]["shards"]
        cover = [np.zeros(n, dtype=int) for n in nw]
        loads = []
        for sh in shards:
            load = 0
            for sym, w0, k in sh["pieces"]:
                cover[sym][w0:w0 + k] += 1
                load += k * cost[sym]
            loads.append(load)
            assert sh["windows"] == sum(p[2] for p in sh["pieces"])
        assert all((c == 1).all() for c in cover)
        assert max(loads) - min(loads) <= 2 * max(cost)
        cuts = {}
        for sh in shards:
            for sym, _, _ in sh["pieces"]:
                cuts[sym] = cuts.get(sym, 0) + 1
        assert max(cuts.values()) <= g


def test_split_symbols_unit():
    for g in (1, 2, 3, 5, 8):
        costs, nwins = [3, 1, 7, 2], [10, 0, 5, 9]
        seen = [[0] * n for n in nwins]
        for r in range(g):
            for i, w0, k in sharding.split_symbols(costs, nwins, g, r):
                for j in range(w0, w0 + k):
                    seen[i][j] += 1
        assert all(all(v == 1 for v in row) for row in seen)


def test_bench_world_size_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r, lines = _bench_line("--gpus", "2", "--plan-only", env=env)
    assert r.returncode != 0 and not lines and "WORLD_SIZE=1" in r.stderr


def test_bench_gpus8_c4_strong_plan():
    """The driver's 8-GPU shape (--gpus 8 --config c4 --scaling strong) rehearsed on a real 8-rank gloo
    rendezvous without a GPU: contiguous window ranges covering the 1,048,576 windows exactly once, each
    rank's series slice = its windows plus the N - hop halo, neighbours overlapping by exactly the halo."""
    r, lines = _bench_line("--gpus", "8", "--config", "c4", "--scaling", "strong", "--plan-only")
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = lines
    shards = line["shards"]
    assert line["n_gpus"] == 8 and [s["rank"] for s in shards] == list(range(8))
    n, hop, W = 2048, 1, 1048576
    assert sum(s["windows"] for s in shards) == W and shards[0]["w0"] == 0
    for a, b in zip(shards, shards[1:]):
        assert b["w0"] == a["w0"] + a["windows"]
        assert a["series"][1] - b["series"][0] == n - hop
    for s in shards:
        assert s["windows"] == W // 8 and s["seed"] == 13  # one batch (same series) split evenly
        assert s["series"] == [s["w0"] * hop, (s["w0"] + s["windows"] - 1) * hop + n]


def test_bench_gpus8_c5_and_weak_plans():
    """C5 over 8 ranks (whole symbols, balanced by output bytes within 10 %) and the weak-scaling north star
    (every rank a full 65536-window batch of its own seed)."""
    r, lines = _bench_line("--gpus", "8", "--config", "c5", "--scaling", "strong", "--c5-shard", "symbols",
                           "--plan-only")
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = lines
    syms = sorted(s for sh in line["shards"] for s in sh["symbols"])
    assert syms == list(range(28))
    lens = (512, 1024, 2048, 4096)
    out_bytes = [sum((20000 - lens[s // 7] + 1) * lens[s // 7] // 2 for s in sh["symbols"]) for sh in line["shards"]]
    assert min(out_bytes) > 0 and max(out_bytes) / min(out_bytes) < 1.10
    r, lines = _bench_line("--gpus", "8", "--config", "north_star", "--plan-only")
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = lines
    assert line["scaling"] == "weak"
    assert [s["windows"] for s in line["shards"]] == [65536] * 8
    assert len({s["seed"] for s in line["shards"]}) == 8
