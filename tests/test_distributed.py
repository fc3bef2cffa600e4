"""Multi-rank paths (world_size 2, 127.0.0.1 rendezvous).

CPU (gloo): a pulse-area scan sharded over ranks through the CPU oracle and gathered to rank 0; the device-buffer
gather (scan.gather_tensor: point-to-point to rank 0 of ragged complex blocks) against a local concatenation.
GPU (gloo, two processes on the one GPU of the box): the bench's two-time sweep with its t1 grid sharded over the
ranks (bench.py --shard t1), each rank propagating its block through libpqd (the batched kernel),
gathered with scan.gather_tensor and compared bit for bit with one process propagating the whole grid."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from pyaceqd_amd.scan import all_gather_tensor, gather_blocks, gather_tensor, run_sharded, shard_range


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


def _gather_worker(rank, world, port, q):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 3 + 4 * rank  # ragged blocks
    x = torch.arange(n, dtype=torch.float64) * (1 + 1j) + 100 * rank
    y = gather_tensor(x.to(torch.complex128), dist, dst=0)
    z = all_gather_tensor(x.to(torch.complex128), dist)
    q.put((rank, (None if y is None else y.numpy(), z.numpy())))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_tensor_ragged_complex_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = np.concatenate([np.arange(3 + 4 * r) * (1 + 1j) + 100 * r for r in range(2)])
    assert np.array_equal(got[0][0], ref)  # gathered to rank 0 only
    assert got[1][0] is None
    assert np.array_equal(got[0][1], ref) and np.array_equal(got[1][1], ref)  # all_gather_tensor: on every rank


N_T1, N_TAU, CHI = 16, 60, 16


def _t1_block_worker(rank, world, port, q):
    try:
        import bench
        from pyaceqd_amd import _lib, engine, scan
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lo, hi = scan.shard_range(N_T1, rank, world)
        sysd, grid, pt, rho0, ops, tr = bench.build_workload(hi - lo, N_TAU, CHI, t1_offset=lo)
        plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt, ctx=_lib.context(0))
        plan.execute()
        path = plan.info()[0]
        y = gather_tensor(plan.output_tensor(device="cpu"), dist)
        if rank == 0:
            q.put(("ok", path, y.numpy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of leaving the peer in its collective
        q.put(("err", rank, repr(e)))
        raise


@pytest.mark.gpu
def test_gloo_world2_t1_sharded_sweep_matches_single_process(monkeypatch):
    monkeypatch.setenv("PQD_SPLIT", "0")  # the batched kernel on both ranks and in the single process
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_t1_block_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    msg = q.get(timeout=100)
    if msg[0] != "ok":
        for p in procs:
            p.kill()
        pytest.fail(f"rank {msg[1]}: {msg[2]}")
    _, path, got = msg
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert path == "batched lock-step sweep"
    import bench
    from pyaceqd_amd import engine
    sysd, grid, pt, rho0, ops, tr = bench.build_workload(N_T1, N_TAU, CHI)
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    ref = np.concatenate([r.ravel() for r in plan.download()])
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)


def test_triangular_rows_balance_the_pairs():
    from pyaceqd_amd.scan import triangular_rows
    for n_t in (0, 1, 5, 128, 1000):
        for w in (1, 2, 3, 8):
            b = [triangular_rows(n_t, r, w) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n_t
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            pairs = [sum(n_t - i for i in range(lo, hi)) for lo, hi in b]
            assert sum(pairs) == n_t * (n_t + 1) // 2
            if n_t >= 8 * w:
                # every rank within one row (at most n_t pairs) of the even share
                assert max(abs(p - n_t * (n_t + 1) / 2 / w) for p in pairs) <= n_t


def _ft8_inputs(n_t=24, dim=3, seed=5):
    rng = np.random.default_rng(seed)
    N2 = dim * dim
    n_map = 2 * n_t + 6
    mk = lambda n: np.asfortranarray((np.eye(N2)[None] + 2e-2 * (rng.normal(size=(n, N2, N2))  # noqa: E731
                                                                + 1j * rng.normal(size=(n, N2, N2)))).transpose(1, 2, 0))
    dm1, dm2 = mk(n_map), mk(n_map)
    precalc = np.asfortranarray(np.stack([np.linalg.matrix_power(dm1[:, :, -1], 2 ** b) for b in range(8)], axis=2))
    rho0 = np.zeros(N2, complex)
    rho0[0] = 1
    ops = [np.asfortranarray(rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim))) for _ in range(8)]
    dt = 0.1
    t1 = dt * np.arange(n_t)
    return (dm1, dm2, rho0, t1, precalc, dt, dim, *ops, False, False, dt * (n_map - 2))


def _ft8_worker(rank, world, port, q):
    try:
        import torch  # noqa: F401
        from pyaceqd_amd.timebin.timebin_tl import four_time_8op_sharded
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        got = four_time_8op_sharded(*_ft8_inputs(), dist=dist)
        if rank == 0:
            q.put(("ok", got))
        else:
            assert got is None
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        q.put(("err", rank, repr(e)))
        raise


def _spawn2(target):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    msg = q.get(timeout=180)
    if msg[0] != "ok":
        for p in procs:
            p.kill()
        pytest.fail(f"rank {msg[1]}: {msg[2]}")
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return msg[1]


@pytest.mark.gpu
def test_gloo_world2_four_time_8op_triangular_split_matches_single_process():
    """the pair triangle of four_time_8op split over two ranks by scan.triangular_rows (two processes on the one GPU),
    gathered to rank 0: bit-identical to one process computing every row"""
    from pyaceqd_amd.timebin.timebin_tl import four_time_8op
    got = _spawn2(_ft8_worker)
    ref = four_time_8op(*_ft8_inputs())
    assert np.array_equal(got, ref)
    assert np.count_nonzero(ref) == 24 * 25 // 2


def _c5_worker(rank, world, port, q):
    try:
        import tempfile
        from tests.test_gpu_c5 import BXS, E0S, _point, _pt
        from pyaceqd_amd.pol_entanglement.G2 import densitymatrix_reuse_scan_sharded
        from pyaceqd_amd.six_level_system.linear import sixls_linear
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pt = _pt()
        with tempfile.TemporaryDirectory() as td:
            insts = [_point(sixls_linear, e0, pt, td) for e0 in E0S for bx in BXS]
            got = densitymatrix_reuse_scan_sharded(insts, [{"bx": bx} for e0 in E0S for bx in BXS], return_rho=True,
                                                   dist=dist)
        if rank == 0:
            q.put(("ok", got))
        else:
            assert got is None
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        q.put(("err", rank, repr(e)))
        raise


@pytest.mark.gpu
def test_gloo_world2_c5_scan_sharded_matches_single_process(tmp_path):
    """BASELINE config 5's tomography scan sharded over two ranks (a contiguous block of grid points
    per rank, two processes on the one GPU), (concurrence, rho) gathered to rank 0: equal to the scan in one process
    to rounding (a two-point launch may take other, parity-tested, kernel paths than the four-point one: the trunk
    pre-pass and split-group choices depend on the batch)"""
    from tests.test_gpu_c5 import BXS, E0S, _point, _pt
    from pyaceqd_amd.pol_entanglement.G2 import densitymatrix_reuse_scan
    from pyaceqd_amd.six_level_system.linear import sixls_linear
    got = _spawn2(_c5_worker)
    pt = _pt()
    insts = [_point(sixls_linear, e0, pt, tmp_path) for e0 in E0S for bx in BXS]
    ref = densitymatrix_reuse_scan(insts, [{"bx": bx} for e0 in E0S for bx in BXS], return_rho=True)
    assert len(got) == len(ref) == 4
    for (cg, rg), (cr, rr) in zip(got, ref):
        assert abs(cg - cr) < 1e-12
        assert np.max(np.abs(rg - rr)) <= 1e-12 * np.max(np.abs(rr))
