"""bench.py's own N-rank launcher: `--gpus N` without
WORLD_SIZE starts N rank processes before any GPU call; a WORLD_SIZE that
disagrees with --gpus exits non-zero.  Rehearsed with --dry-run (gloo
rendezvous, no GPU work) at world sizes 1, 2 and 3."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_launcher_starts_n_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run"])
    assert r.returncode == 0, r.stderr
    # (gloo itself prints "[Gloo] Rank i is connected ..." lines)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 alone prints, once
    d = json.loads(lines[0])
    assert d["dry_run"] is True
    assert d["n_gpus"] == n and d["gpus_arg"] == n
    assert d["ranks"] == list(range(n))
    assert len(set(d["pids"])) == n            # one process per rank
    assert d["max_rank"] == float(n - 1)


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "3", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
    assert r.stdout.strip() == ""


def test_failing_rank_stops_the_launch():
    # rank 1 exits before the rendezvous; rank 0 would wait for it forever,
    # so the launcher must stop rank 0 and report rank 1's status
    r = _run(["--gpus", "2", "--dry-run"], {"TNS_DRYRUN_FAIL_RANK": "1"}, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "rank 1 exited with 3" in r.stderr
    assert "{" not in r.stdout


def test_profiler_preload_detection():
    sys.path.insert(0, str(ROOT))
    import bench
    assert bench.profiler_preloaded({"LD_PRELOAD": "/opt/rocm/lib/librocprofiler-sdk-tool.so"})
    assert not bench.profiler_preloaded({"LD_PRELOAD": "/usr/lib/libfoo.so"})
    assert not bench.profiler_preloaded({})


def test_sigterm_to_launcher_stops_the_ranks(tmp_path):
    """A timeout (SIGTERM) of the launcher must not leave ranks behind."""
    import signal
    import time
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["TNS_DRYRUN_HANG_DIR"] = str(tmp_path)
    p = subprocess.Popen([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dry-run"],
                         env=env)
    deadline = time.time() + 120
    while time.time() < deadline and len(list(tmp_path.glob("rank*"))) < 2:
        time.sleep(0.2)
    pids = [int(f.read_text()) for f in tmp_path.glob("rank*")]
    assert len(pids) == 2
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=60) != 0
    for pid in pids:   # each rank was terminated and reaped by the launcher
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)
