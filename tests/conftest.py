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


def fsm_commands(count, seed, H=10):
    """Synthetic commands (config-4 states) whose four legs carry the phases and FSM states of the reference's leg
    FSMs after a random walk of MPC ticks with early touchdowns (oracle/fsm.py): the per-leg phases differ and some are
    negative (LeggedContactFSM.cpp:61-66,214-221).  -> (ctypes LmpcCommand array, list of the four FSMs per command)."""
    from legged_mpc_control_amd import synth
    from oracle import fsm as F

    rng = np.random.default_rng(seed)
    cmds = synth.commands(synth.config_cfg(4), count, synth.BASE_SEED + 4, first_index=500 + seed)
    fsms = []
    for b in range(count):
        gait = int(rng.integers(0, 3))  # trot, crawl, trot with stand (a stand never swings)
        fs = F.random_walk(rng, gait, 4.0, ticks=int(rng.integers(1, 200)))
        c = cmds[b]
        c.gait, c.gait_speed = gait, 4.0
        for j in range(4):
            c.gait_phase[j] = fs[j].phase
            c.plan_contacts[j] = fs[j].s
        fsms.append(fs)
    return cmds, fsms
