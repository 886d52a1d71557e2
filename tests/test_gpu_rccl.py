"""RCCL on the device path of the frame gather (dist.gather_frames with
backend "nccl", device tensors: no host staging). The pool's boxes have one
GPU and RCCL refuses two ranks on one device, so the N > 1 runs are the
driver's; this test runs the same collective code on a one-rank RCCL
communicator over device frames (the device-tensor branch had
never executed), in a child process so its process group stays its own."""
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

CHILD = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["PSRT_ROOT"])
from petershirleyraytracer_amd import dist as D
dist.init_process_group("nccl", rank=0, world_size=1)
assert dist.get_backend() == "nccl"
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
frames = torch.randint(0, 256, (3, 7, 40, 3), dtype=torch.uint8, device=dev)
out = D._gather_blocks(frames, 7, 0, 1, 0)
torch.cuda.synchronize()
assert out.device.type == "cuda" and torch.equal(out, frames)
acc = torch.randn((2, 5, 16, 3), dtype=torch.float64, device=dev)
out = D._gather_blocks(acc, 5, 0, 1, 0)
assert torch.equal(out.view(torch.int64), acc.view(torch.int64))
dist.destroy_process_group()
print("rccl gather ok")
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_gather_on_device_frames():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               PSRT_ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0 and "rccl gather ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
