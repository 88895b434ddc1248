"""bench.py's rank launch: `python bench.py --gpus N` starts N ranks
itself before any GPU call, every rank checks the group's size against --gpus, and a launcher
whose WORLD_SIZE disagrees with --gpus is refused.  CPU only (--launch-check: gloo, no GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True,
                          timeout=240, env=env, cwd=ROOT)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_gpus_n_starts_n_ranks(n):
    r = _run(["--gpus", str(n), "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout           # one JSON line, from rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "2", "--launch-check"],
             env_extra={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=3 but --gpus 2" in r.stderr
    assert not r.stdout.strip()


def test_rank_command_is_one_process_per_gpu():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.rank_command(8, ["--gpus", "8", "--steps", "5"], 29999)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-3:] == ["--gpus", "8", "--steps", "5"][-3:]
    with pytest.raises(SystemExit):
        bench.check_world(8, "4")
    bench.check_world(8, "8")
    bench.check_world(1, None)
