"""bench.py --gpus N launches its N ranks itself (startmpi's role under mpirun,
src/mpires.f90:21-37): one fresh child process per GPU with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT, rank 0's JSON line on stdout, a non-zero exit
when any rank fails.  Exercised on the CPU through the hidden --dry-run modes (no
GPU, no torch.cuda): `env` (each rank reports its environment), `gloo` (the ranks
join one gloo group over the launcher's rendezvous and rank 0 reports all of them),
`fail` (rank 1 exits with 3 while rank 0 waits: the launcher must end rank 0)."""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(*args, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=env)


def test_launcher_gives_every_rank_its_environment():
    p = _run("--gpus", "3", "--dry-run", "env")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0's line only on stdout
    me = lines[0]["rank"]
    assert me["RANK"] == "0" and me["LOCAL_RANK"] == "0" and me["WORLD_SIZE"] == "3"
    assert me["MASTER_ADDR"] == "127.0.0.1" and int(me["MASTER_PORT"]) > 0
    others = [json.loads(x) for x in p.stderr.splitlines() if x.startswith("{")]
    assert sorted(o["rank"]["RANK"] for o in others) == ["1", "2"]
    assert len({o["rank"]["pid"] for o in others} | {me["pid"]}) == 3  # three processes


def test_launcher_ranks_join_one_gloo_group():
    p = _run("--gpus", "4", "--dry-run", "gloo")
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 4
    ranks = line["ranks"]
    assert [r["RANK"] for r in ranks] == ["0", "1", "2", "3"]
    assert [r["LOCAL_RANK"] for r in ranks] == ["0", "1", "2", "3"]
    assert len({r["MASTER_PORT"] for r in ranks}) == 1 and len({r["pid"] for r in ranks}) == 4


def test_launcher_fails_when_a_rank_fails_and_ends_the_others():
    t0 = time.time()
    p = _run("--gpus", "2", "--dry-run", "fail", timeout=60)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert time.time() - t0 < 40  # rank 0 (sleeping 120 s) was ended, not waited for
    assert "rank 1 exited with 3" in p.stderr


def test_launcher_times_out():
    p = _run("--gpus", "2", "--dry-run", "fail", "--launch-timeout", "0", timeout=60)
    assert p.returncode != 0
