"""bench.py's launch contract on CPU: `--gpus N` without a launcher starts N ranks
itself (a torch.distributed.run child, before any GPU call), the ranks agree on
the world size, and a launcher/flag mismatch fails instead of silently timing
one GPU.  --dry-run stops after rank bring-up (gloo), so no GPU is touched."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    e.update(env or {})
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        if not env or k not in env:
            e.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=240, env=e, cwd=ROOT)


def _last_json(out):
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


def test_gpus2_self_launches_two_ranks():
    p = _run(["--gpus", "2", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    j = _last_json(p.stdout)
    assert j["dry_run"] and j["n_gpus"] == 2 and j["ranks"] == [0, 1] and j["world_sizes_seen"] == [2]


def test_gpus1_dry_run_is_single_rank():
    p = _run(["--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert _last_json(p.stdout)["n_gpus"] == 1


def test_launcher_mismatch_fails_loudly():
    p = _run(["--gpus", "2", "--dry-run"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=1" in (p.stderr + p.stdout)


def test_config5_forward_replicas_dry_run():
    """BASELINE configs[4] (cfg5): forward-only replicas, one view per rank at distinct
    yaws, no collective on the data path; the ranks come up and agree (no GPU)."""
    p = _run(["--config", "5", "--gpus", "2", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    j = _last_json(p.stdout)
    assert j["config"] == 5 and "replicas" in j["mode"] and "no collective" in j["mode"]
    assert j["n_gpus"] == 2 and j["ranks"] == [0, 1] and j["world_sizes_seen"] == [2]
    assert j["yaws"] == [-20.0, 20.0]
    p1 = _run(["--dry-run"])
    assert _last_json(p1.stdout)["config"] == 3


def test_config1_and_config2_dry_run():
    """BASELINE configs[0] (cfg1: fwd+bwd) and configs[1] (cfg2: forward-only
    replicas) are bench.py lines too."""
    for cfg, mode in ((1, "fwd+bwd"), (2, "replicas")):
        p = _run(["--config", str(cfg), "--dry-run"])
        assert p.returncode == 0, p.stderr[-2000:]
        j = _last_json(p.stdout)
        assert j["config"] == cfg and mode in j["mode"]
