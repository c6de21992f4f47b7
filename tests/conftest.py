import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

DIST_OUT = os.path.join(REPO, "gpurun_out", "dist_world2.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device; run with -m gpu on the GPU box")


def _gpu_session(config):
    expr = (config.getoption("markexpr") or "").replace(" ", "")
    return "gpu" in expr and "notgpu" not in expr


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def pytest_sessionstart(session):
    """GPU sessions: run the world-2 class-level sharding check (tests/dist_worker.py) as two
    child processes NOW, before this process initialises the GPU -- a process that has touched
    the GPU must not start other programs. tests/test_gpu_dist.py asserts on its result."""
    config = session.config
    config._wam_dist = None
    if not _gpu_session(config):
        return
    os.makedirs(os.path.dirname(DIST_OUT), exist_ok=True)
    if os.path.exists(DIST_OUT):
        os.remove(DIST_OUT)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "tests", "dist_worker.py"), DIST_OUT]
    try:
        p = subprocess.run(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=600)
        log = p.stdout.decode(errors="replace")[-4000:]
        res = json.load(open(DIST_OUT)) if os.path.exists(DIST_OUT) else None
        config._wam_dist = {"rc": p.returncode, "log": log, "result": res}
    except subprocess.TimeoutExpired as e:
        config._wam_dist = {"rc": -1, "log": "timeout: %s" % e, "result": None}


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")


@pytest.fixture(scope="session")
def dist_world2(request):
    return request.config._wam_dist
