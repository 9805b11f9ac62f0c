"""GPU, two ranks on one device (gloo collectives on device tensors): the sharded brax and
gym paths with the HIP kernels equal the single-process batch (scripts/multirank_check.py;
the 8-GPU RCCL run uses the same script with --backend nccl)."""
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
    assert "brax True gym True key True" in r.stdout
