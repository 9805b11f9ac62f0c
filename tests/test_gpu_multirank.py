"""GPU, two ranks on one device (gloo collectives on device tensors) and one rank over RCCL:
the sharded brax and gym paths and the overlapped obs gather with the HIP kernels equal the
single-process batch (scripts/multirank_check.py; the 8-GPU RCCL run uses the same script with
--backend nccl)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("name", ["ant_tag", "ant_heavenhell"])
def test_two_ranks_one_gpu_equal_single(name):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "scripts", "multirank_check.py"), "--backend", "gloo", "--env", name]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=200)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0
    assert "brax True gym True key True gather True" in r.stdout


@pytest.mark.parametrize("name", ["ant_heavenhell"])
def test_rccl_world1_product_path(name):
    """The same check over RCCL (backend nccl) with one rank: the process group, the sharded
    brax and gym chains' collectives (the gym path's any-done all-reduce) and ObsGatherer's
    side-stream all-gather run through RCCL on the device.  (RCCL refuses two ranks on one
    device -- "Duplicate GPU detected", profiles/r7v -- so world 2 runs over gloo above and
    the 8-GPU node is the first place RCCL sees more than one rank.)"""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "scripts", "multirank_check.py"), "--backend", "nccl", "--env", name]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=200)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0
    assert "world=1 backend=nccl: brax True gym True key True gather True" in r.stdout


def test_rccl_world1_gym_graph_capture():
    """The sharded gym step's any-done all-reduce captured into the hipGraph with the kernels
    (rollout.GymGraphRollout over RCCL): two replays of 8 captured steps equal 16 eager steps
    bit for bit -- obs, reward, done and the gym key (every env ends an episode on the way)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "scripts", "gym_capture_check.py"), "--backend", "nccl"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=200)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0
    assert "world=1 rank=0 backend=nccl: obs True reward True done True key True" in r.stdout
