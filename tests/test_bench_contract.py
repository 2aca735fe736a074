"""bench.py host logic (CPU): workload table vs BASELINE.json, FLOP accounting, PMC lookup."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_default_workload_is_the_metric_config(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.gpus, a.workload, a.batch_per_gpu, a.alg, a.dtype, a.seq_mult) == (1, "c2", 32, "ddpm", "bf16", 1)
    assert a.respacing == ""


def test_workloads_follow_baseline_configs():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert "frames" in json.dumps(base).lower()
    w = bench.WORKLOADS
    assert w["c4"]["seq_mult"] == 4 and w["c4"]["dtype"] == "fp8"
    assert w["c5"]["alg"] == "ddim" and w["c5"]["respacing"] == "ddim50" and w["c5"]["batch_per_gpu"] == 128
    assert not w["c2"]["overlap"] and not w["c5"]["overlap"]  # the clip-pair C5 loop fills the chip


def test_clip_step_flops_hand_count():
    L, Tm, d, C, layers = 40, 32, 256, 123, 4
    # per layer: QKV 3d^2, SA out d^2, CA Q d^2, CA out d^2, FFN 2 x 4d^2 (rows L); emb C->d, out d->C
    gemm = 2 * L * (C * d + d * C + layers * 14 * d * d)
    attn = layers * 4 * L * (L + Tm) * d
    conv = layers * 4 * 6 * L * d
    # the step token's per-step memory work: step MLP 2 x d^2, emb_mem row 0, per layer K and V of
    # memory rows 0 and 1
    step = 2 * 2 * d * d + 2 * d * d + layers * 2 * 2 * (2 * d * d)
    assert bench.clip_step_flops(L, Tm, d, C, layers) == gemm + attn + conv + step
    assert abs(bench.clip_step_flops(L, Tm, d, C, layers) / 1e6 - 314.3) / 314.3 < 2e-3
    # C1's two-way decoder: GEMMs + attention = SURVEY.md 8d's 11,839.6 MFLOP
    tw = bench.twoway_clip_step_flops(34, 104, 512, 126, 10)
    conv2 = 10 * 6 * 3 * 512 * (34 + 104 + 138)
    assert abs((tw - conv2) / 1e6 - 11839.6) < 0.1


@pytest.mark.parametrize("workload,prefix", [("c2", "mr_kernel"), ("c5", "psk_kernel")])
def test_pmc_traffic_reads_committed_summary(workload, prefix):
    tr = bench.pmc_traffic(prefix, workload)
    assert tr is not None and os.path.exists(os.path.join(ROOT, tr["source"]))
    if tr.get("stale"):   # taken on other kernel sources: reported as stale, never as this code's traffic
        assert "bytes_per_launch" not in tr and tr["summary_csrc"] != tr["current_csrc"] == bench.csrc_hash()
    else:
        assert tr["bytes_per_launch"] == tr["read"] + tr["write"] > 0
    assert bench.pmc_traffic(prefix, "nope") is None


def test_launch_command_one_rank_per_gpu():
    cmd = bench.launch_command(["--gpus", "4", "--steps", "3"], 4, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-port=29555" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "3"]


def _rehearse(n, *extra):
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("RANK", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--rehearse", *extra],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints the only line
    return json.loads(lines[0])


def test_self_launch_rehearsal_matches_single_rank():
    """bench.py --gpus N spawns N ranks itself (no external torchrun); over gloo with the oracle
    sampler, the all-gathered clips equal a single rank's bit for bit."""
    one = _rehearse(1)
    for n in (2, 3):
        res = _rehearse(n)
        assert res["rehearsal"] and res["world"] == n and res["global_batch"] == 2 * n
        assert res["shape"] == [2 * n, 123, 40]
        assert res["first"][:2] == one["first"]  # global clips 0, 1: same wav rows, same noise keys
        d = res["distributed"]   # the fields a GPU run at N > 1 reports (max over ranks)
        assert d["backend"] == "gloo" and d["world_size"] == n
        assert d["all_gather_bytes"] == 2 * n * 123 * 40 * 4
        assert d["all_gather_ms_max_over_ranks"] >= 0.0
    assert one["distributed"] is None


def test_rehearsal_at_the_c5_eight_gpu_shape():
    """C5's 8-GPU leg (BASELINE.json configs[4]: B = 1024 over 8 ranks, 128 clips each) through the
    same launch / shard / all-gather path over gloo: the gathered payload is SURVEY.md 8e's 2.52 MB
    per rank, 20.2 MB in all, and the clips come back in global order (equal to one rank's)."""
    one = _rehearse(1, "--workload", "c5", "--batch-per-gpu", "1024")
    eight = _rehearse(8, "--workload", "c5")
    assert eight["global_batch"] == one["global_batch"] == 1024 and eight["shape"] == [1024, 123, 40]
    d = eight["distributed"]
    assert d["world_size"] == 8 and d["backend"] == "gloo"
    assert d["all_gather_bytes_per_rank"] == 128 * 123 * 40 * 4 == 2_519_040
    assert d["all_gather_bytes"] == 8 * 2_519_040 == 20_152_320
    assert eight["first"] == one["first"] and eight["checksum"] == one["checksum"]


def test_headline_pmc_summary_matches_the_kernel_sources():
    """The default (driver-run) C2 line prices its roofline traffic from a PMC summary taken on THIS
    csrc/ tree: a kernel change has to come with a fresh summary (scripts/pmc_all.sh)."""
    tr = bench.pmc_traffic("mr_kernel", "c2")
    assert tr is not None and not tr.get("stale"), tr
    assert tr["bytes_per_launch"] > 0


class _FakeLib:
    """The ggd_* calls workload_subrecord makes, answering like a loop that ran (kind, avg us)."""

    def __init__(self, kind, avg_us, launches):
        self.kind, self.avg_us, self.launches, self.prof, self.calls = kind, avg_us, launches, [], None

    def ggd_set_route(self, h, knob, value):
        return 0

    def ggd_set_profiling(self, h, on):
        self.prof.append(on)
        if self.calls is not None:
            self.calls.append(("prof", on))
        return 0

    def ggd_kernel_time(self, h, which, avg, cnt):
        avg._obj.value, cnt._obj.value = self.avg_us, self.launches
        return 0

    def ggd_profile_kind(self, h):
        return self.kind


@pytest.mark.parametrize("workload,kind,avg_us,launches", [("c4", 5, 159000.0, 1), ("c5", 4, 7500.0, 1)])
def test_workload_subrecord_fields(monkeypatch, workload, kind, avg_us, launches):
    """The C4 / C5 sub-records of the default C2 line: frames/s over the timed passes, ms per pass,
    the loop's hipEvent time and its roofline fraction from SURVEY.md 8d's FLOPs (fp8 peak for C4's
    block-scaled MFMA, bf16 for C5)."""
    import types
    import torch as th
    import __graft_entry__ as ge
    pkg = ge.load_package()
    monkeypatch.setattr(th.cuda, "synchronize", lambda *a, **k: None)
    w = bench.WORKLOADS[workload]
    L = 40 * w["seq_mult"]
    lib = _FakeLib(kind, avg_us, launches)
    calls = []
    lib.calls = calls

    class FakeModel:
        arch = {"d_model": 256, "n_layers": 4}
        _ctx = {0: types.SimpleNamespace(lib=lib, h=None, desc=types.SimpleNamespace(speech_len=31 if L == 40 else 126))}

        def load_state_dict(self, sd):
            pass

        def sync(self):
            calls.append("sync")

        def _release(self):
            calls.append("release")

    class FakeDiffusion:
        num_timesteps = 50 if w["respacing"] else 1000

        def _loop(self, model, shape, model_kwargs, seed, extras):
            calls.append(shape)
            return {"sample": th.zeros(shape)}
        p_sample_loop = ddim_sample_loop = _loop

    monkeypatch.setattr(pkg, "create_model", lambda *a, **k: (FakeModel(), FakeDiffusion(), None, None, None))
    monkeypatch.setattr(pkg, "create_diffusion", lambda *a, **k: FakeDiffusion())
    monkeypatch.setattr(pkg, "init_state_dict", lambda *a, **k: {})
    passes = 3 if workload == "c5" else 1
    rec = bench.workload_subrecord(pkg, workload, th.device("cpu"), passes=passes)
    assert calls.count((w["batch_per_gpu"], 123, L)) == passes + 2 and calls[-1] == "release"
    assert lib.prof == [1, 0]   # one profiled pass, after the timed ones
    shape = (w["batch_per_gpu"], 123, L)
    # warm-up, the timed passes, their sync; then the profiled pass alone between the profiling calls
    assert calls == [shape] * (1 + passes) + ["sync", ("prof", 1), shape, "sync", ("prof", 0), "release"]
    for k in ("workload", "value", "unit", "ms_per_step", "steps", "kernel", "kernel_avg_launch_us",
              "roofline_frac", "peak_tflops", "flop_per_launch"):
        assert k in rec, k
    assert rec["unit"] == "frames/s" and rec["steps"] == passes and rec["value"] > 0
    T = FakeDiffusion.num_timesteps
    flop = bench.clip_step_flops(L, 1 + FakeModel._ctx[0].desc.speech_len, 256, 123, 4) * w["batch_per_gpu"] * T
    assert rec["flop_per_launch"] == flop
    peak = bench.FP8_PEAK_TFLOPS if workload == "c4" else bench.BF16_PEAK_TFLOPS
    assert rec["peak_tflops"] == peak
    assert abs(rec["roofline_frac"] - flop / (avg_us * 1e-6) / 1e12 / peak) < 1e-6
    assert rec["dtype"] == ("fp8" if workload == "c4" else "bf16")
