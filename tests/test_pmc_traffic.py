"""bench.py's own PMC passes (scripts/pmc_traffic.py): the child command, the per-step arithmetic and the
fallback when rocprofv3 is unavailable -- CPU only, no profiler run."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "scripts"))
import pmc_traffic  # noqa: E402

import bench  # noqa: E402


def _rows(counter, kernels):
    return [{"Counter_Name": counter, "Kernel_Name": k, "Counter_Value": str(v)} for k, v in kernels]


def test_summarize_per_step_with_prepass():
    """C3-like step: a Kalman pre-pass plus the spectrum launch; FETCH doubled (gfx950), WRITE as is."""
    f = _rows("FETCH_SIZE", [("void wsp::kcore::kalman_pk2_kernel<32>(...)", 1000.0),
                             ("void wsp::core::spectrum_kernel<float>(...)", 500.0)] * 3
              + [("at::native::elementwise_kernel", 99999.0)])
    w = _rows("WRITE_SIZE", [("void wsp::kcore::kalman_pk2_kernel<32>(...)", 1024.0),
                             ("void wsp::core::spectrum_kernel<float>(...)", 512.0)] * 3)
    r = pmc_traffic.summarize(f, w, "c3", "c3")
    assert r["read_bytes_corrected"] == 1500.0 * 1024 * 2
    assert r["write_bytes"] == 1536.0 * 1024
    assert r["hbm_bytes_per_launch"] == r["read_bytes_corrected"] + r["write_bytes"]


def test_summarize_missing_pass():
    assert "hbm_bytes_per_launch" not in pmc_traffic.summarize([], [], "north_star", "north_star")


def test_bench_key():
    assert pmc_traffic.bench_key("c4", "fft", 0) == "c4_fft"
    assert pmc_traffic.bench_key("c3", "auto", 8) == "c3_v8"
    assert pmc_traffic.bench_key("c5", "auto", 0, "plans") == "c5_plans"
    assert pmc_traffic.bench_key("north_star") == "north_star"


def test_run_pmc_child_command(monkeypatch):
    """The child runs the same configuration for 3 steps without the CPU baseline, settle or PMC of its own."""
    seen = {}

    def fake(cmd, cfg, key, timeout=120.0):
        seen.update(cmd=cmd, cfg=cfg, key=key)
        return {"hbm_bytes_per_launch": 1.0}

    monkeypatch.setattr(pmc_traffic, "collect", fake)
    argv = ["--config", "c3", "--steps", "50", "--warmup=4", "--variant", "8", "--cpu-seconds", "3", "--pmc", "on"]
    args = bench.parse(argv)
    assert bench.run_pmc(args, argv) == {"hbm_bytes_per_launch": 1.0}
    cmd = seen["cmd"]
    assert cmd[1].endswith("bench.py")
    tail = cmd[2:]
    assert tail[:4] == ["--config", "c3", "--variant", "8"]
    assert tail[4:] == ["--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-settle", "--pmc", "off"]
    assert seen["key"] == "c3_v8"


@pytest.mark.parametrize("argv,env,want", [([], {}, True), (["--no-cpu-baseline"], {}, False),
                                           (["--no-cpu-baseline", "--pmc", "on"], {}, True),
                                           (["--pmc", "off"], {}, False), ([], {"WSP_BENCH_PMC_CHILD": "1"}, False),
                                           (["--emulate-shard", "1/8"], {}, False)])
def test_want_pmc(monkeypatch, argv, env, want):
    monkeypatch.delenv("WSP_BENCH_PMC_CHILD", raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    assert bench.want_pmc(bench.parse(argv)) is want


def test_collect_without_profiler(monkeypatch):
    monkeypatch.setattr(pmc_traffic.shutil, "which", lambda name: None)
    assert pmc_traffic.collect(["true"], "north_star", "north_star") is None
