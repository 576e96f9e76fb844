import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session", autouse=True)
def _built(request):
    """Build the HIP library and the oracle in-tree if they are missing (no-op when built).

    When GPU tests are selected, torch's HIP runtime is brought up first: a selection whose first
    GPU tests drive the C-ABI library alone (ctypes) initialised HIP before torch, and torch then
    reported no device to the later tests that use it (seen with tests/test_gpu_parity.py run first)."""
    from legged_mpc_control_amd import build as B
    from oracle import oracle as O

    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch

        torch.cuda.is_available()
    B.build_native()
    O.build()


def golden_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "golden_*.npz")))


def load_golden(path):
    d = np.load(path, allow_pickle=False)
    from oracle import oracle as O

    pr = d["params"]
    op = O.make_params(pr[0:12], pr[12:24], pr[24], pr[25:34].reshape(3, 3), pr[34], pr[35], pr[36], pr[37])
    return dict(H=int(d["H"]), op=op, params=pr, rec=d["rec"], contact=d["contact"], grf=d["grf"],
                kkt=d["kkt"], n_active=d["n_active"], meta=[str(m) for m in d["meta"]],
                normals=d["normals"] if "normals" in d.files else None)


def lmpc_params_from(pr):
    from legged_mpc_control_amd import LmpcParams

    p = LmpcParams()
    p.q_weights[:] = list(pr[0:12])
    p.r_weights[:] = list(pr[12:24])
    p.robot_mass = float(pr[24])
    p.trunk_inertia[:] = list(pr[25:34])
    p.mu, p.f_max, p.gravity, p.dt = (float(x) for x in pr[34:38])
    return p


def rel_err(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b)) / np.maximum(1.0, np.abs(np.asarray(b)))))
