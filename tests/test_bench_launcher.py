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
