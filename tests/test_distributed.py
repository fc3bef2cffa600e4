"""Multi-rank path on CPU (gloo, world_size 2): a pulse-area scan sharded over ranks, each rank
propagating its block (through the CPU oracle here; on the GPU box the same code drives libpqd),
gathered to rank 0 and compared with the single-process result."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from pyaceqd_amd.scan import gather_blocks, run_sharded, shard_range


def test_shard_range_partitions():
    for n in (0, 1, 7, 256):
        for w in (1, 2, 3, 8):
            blocks = [shard_range(n, r, w) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1


def _work(block):
    import bench
    from oracle import oracle
    out = []
    for e0 in block:
        sysd, grid, pt, rho0, ops, tr = bench.build_workload(2, 30, 16, scan_offset=int(round((e0 - 1.0) / 0.05)))
        r = oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt)
        out.append(np.concatenate([x.ravel() for x in r]))
    return out


def _worker(rank, world, port, units, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = run_sharded(units, _work, dist)
    if rank == 0:
        q.put([np.asarray(x) for x in res])
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_scan_matches_single_process():
    units = [1.0 + 0.05 * k for k in range(5)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, units, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = _work(units)
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)


def test_gather_blocks_single_process_passthrough():
    assert [int(x) for x in gather_blocks([np.array(1), np.array(2)], None)] == [1, 2]
