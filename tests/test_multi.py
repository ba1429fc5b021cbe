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
