"""CPU: ``bench.py --gpus N`` without torchrun starts the N ranks itself (bench.launch_ranks):
each child gets its own RANK / LOCAL_RANK, the shared WORLD_SIZE and a rendezvous on
127.0.0.1 at one free port; a failing rank fails the launch and the others are stopped."""
import json
import os
import sys
import textwrap
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _script(tmp_path, body):
    p = tmp_path / "child.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_launcher_rank_environment(tmp_path):
    import bench
    script = _script(tmp_path, """
        import json, os, sys
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
        r = os.environ["RANK"]
        with open(os.path.join(sys.argv[1], f"rank{r}.json"), "w") as f:
            json.dump({k: os.environ.get(k) for k in keys} | {"argv": sys.argv[2:]}, f)
    """)
    assert bench.launch_ranks(3, argv=[str(tmp_path), "--steps", "5"], script=script) == 0
    envs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"} and {e["LOCAL_WORLD_SIZE"] for e in envs} == {"3"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    ports = {e["MASTER_PORT"] for e in envs}
    assert len(ports) == 1 and 0 < int(ports.pop()) < 65536
    assert all(e["argv"] == ["--steps", "5"] for e in envs)


def test_launcher_failing_rank_stops_the_rest(tmp_path):
    import bench
    script = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(600)  # a rank left waiting at a barrier
    """)
    t0 = time.time()
    assert bench.launch_ranks(2, argv=[], script=script) == 3
    assert time.time() - t0 < 60


def test_launcher_runs_real_bench_parser_world4(capfd):
    """``bench.py --gpus 4 --dry-run``: launch_ranks starts four ranks of the real bench.py,
    each parses the real argument list, joins a gloo process group on 127.0.0.1 and sends its
    row; rank 0 prints one JSON line with all four ranks' devices and shard sizes (ragged:
    65 537 = 16 385 + 3 x 16 384)."""
    import bench
    argv = ["--gpus", "4", "--dry-run", "--env", "ant_tag", "--global-batch", "65537", "--gather-obs",
            "--obs-mask", "no-cfrc", "--steps", "7"]
    env = dict(os.environ)
    os.environ.pop("WORLD_SIZE", None)
    try:
        assert bench.launch_ranks(4, argv=argv) == 0
    finally:
        os.environ.clear()
        os.environ.update(env)
    out = [l for l in capfd.readouterr().out.splitlines() if l.startswith("{")]
    assert len(out) == 1  # rank 0 only
    line = json.loads(out[0])
    assert line["world_size"] == 4 and line["env"] == "ant_tag" and line["steps"] == 7
    assert line["obs_mask"] == "no-cfrc" and line["gather_obs"] is True
    assert [r["rank"] for r in line["per_rank"]] == [0, 1, 2, 3]
    assert [r["envs"] for r in line["per_rank"]] == [16385, 16384, 16384, 16384]
    assert len({r["pid"] for r in line["rank_devices"]}) == 4
    assert all("obs_allgather_ms" in r for r in line["per_rank"])


def test_launcher_bad_argument_fails_every_rank():
    """an argument the real parser rejects fails the launch (exit 2 from argparse)"""
    import bench
    assert bench.launch_ranks(2, argv=["--gpus", "2", "--dry-run", "--env", "no_such_env"]) == 2


def test_launcher_sigterm_stops_the_ranks(tmp_path):
    """SIGTERM to the launching process terminates its ranks (they would otherwise be left
    running, e.g. waiting at a barrier) and it exits 143."""
    import signal
    import subprocess
    child = _script(tmp_path, """
        import os, sys, time
        open(os.path.join(sys.argv[1], "pid%s" % os.environ["RANK"]), "w").write(str(os.getpid()))
        time.sleep(600)
    """)
    parent = subprocess.Popen([sys.executable, "-c", textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {ROOT!r})
        import bench
        sys.exit(bench.launch_ranks(3, argv=[{str(tmp_path)!r}], script={child!r}))
    """)])
    t0 = time.time()
    while len(list(tmp_path.glob("pid*"))) < 3:
        assert time.time() - t0 < 60 and parent.poll() is None
        time.sleep(0.1)
    pids = [int((tmp_path / f"pid{r}").read_text()) for r in range(3)]
    parent.send_signal(signal.SIGTERM)
    assert parent.wait(timeout=60) == 143

    def alive(pid):
        try:
            st = open(f"/proc/{pid}/stat").read().split(")")[-1].split()[0]
        except OSError:
            return False
        return st != "Z"

    t0 = time.time()
    while any(alive(p) for p in pids) and time.time() - t0 < 10:
        time.sleep(0.1)
    assert not any(alive(p) for p in pids)
