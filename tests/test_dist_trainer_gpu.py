"""GPU tier: MaPLeFederated.train()'s distributed branch with the real HIP kernels (trainers/maple_fed.py:247-290).

Two ranks started by torch.distributed.run as a fresh child process (never an exec of this process), both on
the box's GPU with MAPFED_DIST_BACKEND=gloo (RCCL refuses two ranks on one device; the driver's multi-GPU runs
use RCCL, one rank per GPU).  Each rank builds the aggregator as train.py does and runs one federated round;
tests/diagnostics/dist_trainer_check.py then checks every rank's global weights against
oracle.safe_average_weights (the reference's trainers/maple_fed.py:309-315, pinned by tests/golden/fedavg.npz)
of all clients' post-epoch trainables, bit for bit: 2 clients (one per rank) and 4 (two per rank, trained one
after another)."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(420)
@pytest.mark.parametrize("clients", [2, 4])
def test_two_rank_trainer_round_bit_exact_fedavg(dev, tmp_path, clients):
    out = tmp_path / f"dist_{clients}.json"
    env = dict(os.environ, MAPFED_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(ROOT / "tests/diagnostics/dist_trainer_check.py"), "--clients", str(clients), "--out", str(out)]
    res = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         timeout=400)
    assert res.returncode == 0, res.stdout[-4000:]
    verdict = json.loads(out.read_text())
    assert verdict["ok"] and verdict["num_clients"] == clients and len(verdict["ranks"]) == 2
    for r in verdict["ranks"]:
        assert r["n_mismatch"] == 0 and r["valid_clients"] == clients and r["clients_differ"]
        assert len(r["clients"]) == clients // 2
