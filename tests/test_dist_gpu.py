"""The multi-GPU code paths on one GPU (the driver's 8-GPU scaling run must not be their first execution):

* nusiprop_amd.dist.evolve_sharded with Plan.evolve on a world-1 RCCL process group: the device-staged all_gather
  and gather of the flux blocks (dist._gather_blocks' "nccl" branch) run, and the gathered fluxes equal one plain
  Plan.evolve bit for bit;
* bench.py under torch.distributed.run with one rank: init_process_group("nccl", device_id=...), the timing
  barrier and the max-over-ranks all_reduce run, and the line reports the RCCL process group.
Both run as child processes (torch's runtime initialised before libnusi's, as in bench.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    e.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return e, port


def _json(out):
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert out.returncode == 0 and len(lines) == 1, out.stdout[-2000:] + out.stderr[-4000:]
    return json.loads(lines[0])


def test_evolve_sharded_on_rccl_world1():
    env, _ = _env()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "nccl_worker.py")], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=110)
    j = _json(out)
    assert j["backend"] == "nccl" and j["world"] == 1 and j["bitexact"] and j["all_reduce"] == 1.0
    assert j["shape"] == [j["points"], 3, 100]


def test_bench_under_torchrun_one_rank():
    env, _ = _env()
    env.pop("MASTER_ADDR")
    env.pop("MASTER_PORT")
    # --standalone: the rendezvous store binds a port the OS picks (a probed-then-closed port was taken by another
    # process between the probe and torchrun's bind once: EADDRINUSE, gpurun_out/r7a)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1", "--nnodes=1",
           "--nproc-per-node", "1", os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline", "--no-secondary", "--no-parity"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    j = _json(out)
    assert j["n_gpus"] == 1 and j["config"]["process_group"] == "nccl" and j["value"] > 0 and j["invalid_outputs"] == 0
