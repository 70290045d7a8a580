import json
import os
import subprocess
import sys
import tempfile
import uuid

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the gpurun box)")
    config.addinivalue_line("markers", "slow: takes more than a few seconds")


def native_built():
    from amdvgpu.shim.native import LIB_DIR
    return os.path.exists(os.path.join(LIB_DIR, "libvgpu_region.so"))


@pytest.fixture(scope="session", autouse=True)
def _build_native():
    """Builds the native tree once per session (incremental make)."""
    from amdvgpu.shim.native import ensure_built
    rc = ensure_built()
    assert rc == 0, "native build failed"


@pytest.fixture
def region_path(tmp_path):
    return str(tmp_path / f"vgpu-{uuid.uuid4().hex}.cache")


CHILD_PRELUDE = f"""
import json, os, sys, time
sys.path.insert(0, {REPO!r})
def emit(**kw):
    print("RESULT " + json.dumps(kw), flush=True)
"""


def run_child(code, contract=None, preload=True, timeout=600, check=True, extra_env=None):
    """Runs python `code` in a child process as a vGPU 'container'. Returns (results, proc)."""
    from amdvgpu.shim.launcher import apply_contract
    env = apply_contract(contract or {}, preload=preload and contract is not None)
    if extra_env:
        env.update(extra_env)
    p = subprocess.run([sys.executable, "-c", CHILD_PRELUDE + code], env=env, capture_output=True, text=True,
                       timeout=timeout)
    results = [json.loads(l[7:]) for l in p.stdout.splitlines() if l.startswith("RESULT ")]
    if check and p.returncode != 0:
        raise AssertionError(f"child failed rc={p.returncode}\nstdout:\n{p.stdout[-4000:]}\nstderr:\n{p.stderr[-4000:]}")
    return results, p


def spawn_child(code, contract=None, preload=True, extra_env=None):
    from amdvgpu.shim.launcher import apply_contract
    env = apply_contract(contract or {}, preload=preload and contract is not None)
    if extra_env:
        env.update(extra_env)
    return subprocess.Popen([sys.executable, "-c", CHILD_PRELUDE + code], env=env, stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True)


def child_results(stdout):
    return [json.loads(l[7:]) for l in stdout.splitlines() if l.startswith("RESULT ")]


@pytest.fixture
def tmp_region():
    p = os.path.join(tempfile.gettempdir(), f"vgpu-test-{uuid.uuid4().hex}.cache")
    yield p
    if os.path.exists(p):
        os.unlink(p)
