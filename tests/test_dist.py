"""world_size-2 and -4 gloo tests of the multi-rank path (CPU): every rank builds its own
shard from (seed, global index), solves it (here with the oracle standing in for
the device solve), and rank 0 gathers the GRFs point-to-point; the gathered
batch must equal a single-process solve of the global batch, and the bench
bookkeeping collectives (max time, status sums) must reduce correctly."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir, per_rank):
    import sys

    import torch
    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from legged_mpc_control_amd import dist as D
    from legged_mpc_control_amd import synth
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, w, lr = D.env_rank()
    assert (r, w, lr) == (rank, world, rank)
    first, last = D.split_range(r, w, per_rank * w - 1)  # ragged: rank 0 owns one QP less
    p, H, rec, con = synth.config_batch(4, count=last - first, first_index=first)
    grf, status, fails = O.solve_batch(O.params_from(p), H, rec, con, n_threads=1)
    t = D.max_over_ranks(float(rank + 1), dist)
    s = D.sum_over_ranks([float((status == 0).sum()), float(fails)], dist)
    counts = [b - a for a, b in (D.split_range(i, w, per_rank * w - 1) for i in range(w))]
    full = D.gather_to_rank0(torch.from_numpy(grf), dist, w, r, counts=counts)
    if r == 0:
        np.save(os.path.join(out_dir, "gathered.npy"), full.numpy())
        np.save(os.path.join(out_dir, "reduced.npy"), np.array([t] + s))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,per_rank", [(2, 6), (4, 3)])
def test_multi_rank_shard_and_gather(tmp_path, world, per_rank):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), per_rank), nprocs=world, join=True)
    from legged_mpc_control_amd import synth
    from oracle import oracle as O

    p, H, rec, con = synth.config_batch(4, count=world * per_rank - 1)
    ref, status, fails = O.solve_batch(O.params_from(p), H, rec, con, n_threads=2)
    gathered = np.load(tmp_path / "gathered.npy")
    assert gathered.shape == ref.shape
    assert np.array_equal(gathered, ref)
    t, ok, nfail = np.load(tmp_path / "reduced.npy")
    assert t == float(world) and ok == world * per_rank - 1 and nfail == 0


def test_split_range_covers_total():
    from legged_mpc_control_amd import dist as D

    for world in (1, 2, 3, 8):
        spans = [D.split_range(r, world, 65536) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == 65536
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
