"""CPU: bench.py's multi-GPU contract without a GPU (--dry-run: no device work).

`python3 bench.py --gpus N` (WORLD_SIZE unset, the driver's single-command form)
must start N ranks itself, one process per GPU, and report n_gpus = N with the
whole-job global batch; under torch.distributed.run (WORLD_SIZE set) a mismatch
between --gpus and the world size is an error (BASELINE configs[3])."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.parametrize("n", [2, 3])
def test_bench_launches_its_own_ranks(n):
    r = _run(["--gpus", str(n), "--same-device", "--dist-backend", "gloo", "--dry-run", "--steps", "5",
              "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n
    assert d["config"]["global_batch"] == 4096 * n
    assert d["config"]["parallelism"].startswith(f"dp{n}")
    assert d["scaling"] == "weak" and d["steps"] == 5 and d["dry_run"]
    assert d["metric"].startswith("control steps/sec")


def test_bench_world_mismatch_fails():
    r = _run(["--gpus", "4", "--dry-run", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_bench_failing_rank_fails_the_job():
    # ranks that cannot start (here: an RCCL process group on a host without a GPU)
    # must fail the job with a non-zero status, not leave the launcher waiting
    r = _run(["--gpus", "2", "--dry-run", "--steps", "1", "--dist-backend", "nccl"], timeout=120)
    assert r.returncode != 0


def test_traffic_null_when_profile_is_stale(tmp_path, monkeypatch):
    """roofline.traffic comes from the committed --pmc summary only while the kernel
    sources are the ones it was measured on: a summary entry
    with another source digest yields None and says why."""
    sys.path.insert(0, ROOT)
    import bench
    from go2_onnx_controller_amd.provenance import kernel_source_digest
    kern = "policy_mlp_kernel<8, 1, 3, 1, 3, 4>"
    name = f"void go2pi::{kern}(go2pi::DevProgram const*, float const*, float*, int)"
    (tmp_path / "profiles").mkdir()
    summary = tmp_path / "profiles" / "pmc_summary.json"
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    for digest, want in [(kernel_source_digest(), 19.0e6), ("0123456789abcdef", None), (None, None)]:
        entry = {"hbm_bytes_per_launch": 19.0e6, "source": "rXX_mlp512_kernel_stats.csv"}
        if digest:
            entry["src_digest"] = digest
        summary.write_text(json.dumps({"workloads": {"go2_mlp_512_b4096": {name: entry}}}))
        got, note = bench.load_pmc("go2_mlp_512_b4096", kern)
        assert got == want, note
        assert ("stale" in note) == (want is None)
    assert bench.load_pmc("other_workload", kern) == (None, "no committed rocprofv3 --pmc summary of this kernel")
