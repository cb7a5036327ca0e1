"""GPU, two ranks: the multi-GPU path end to end with real device summaries
(SURVEY.md §8e).  Two processes share GPU 0 (the box has one card; RCCL cannot
put two ranks of one communicator on one GPU, so the collective runs over gloo
on host copies -- the C-ABI RCCL form is covered at one rank in
test_gpu_comm.py and at N>1 only by the driver's 8-GPU runs).

Each rank owns its own documents, exactly as bench.py shards them (seed +
(rank << 40)): it generates its config-5-shaped shard on the device, folds
r0 <- r1 <- ... <- r7, checks every document of its fold bit-exactly against
the C oracle, reduces its output version vectors with crdt_causal_context_async
on the device, and all-reduces that summary (u64 max).  The parent checks the
global context against the oracle's max over every document of every rank --
the reference's counterpart is (*VersionVector).Merge applied across all the
merged states (crdt-misc.go:43-55)."""

import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED
N_DOCS, P, E, R = 8192, 8, 16, 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist

        import crdtgpu
        from crdtgpu import CRDT_FOLD_AWSET
        from crdtgpu import dist as cdist
        from crdtgpu.batch import OutBuffers, SrcBuffers
        from oracle import oracle
        from test_gpu_parity import assert_same_all, host_out

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        eng = crdtgpu.Engine(0)
        seed = SEED + (rank << 40)
        D = OutBuffers(N_DOCS, R, N_DOCS * E, device=dev)
        S = SrcBuffers(R, N_DOCS, N_DOCS * (P - 1), N_DOCS * (P - 1) * E, 0, device=dev)
        eng.gen_replicas_async(seed, N_DOCS, P, E, D, S)
        out = OutBuffers(N_DOCS, R, N_DOCS * E * P, device=dev)
        eng.fold_async(CRDT_FOLD_AWSET, D.as_batch(), S, out)
        eng.sync()
        # this rank's fold, every document, vs the oracle
        torch.cuda.synchronize()
        rc, want = oracle.fold(CRDT_FOLD_AWSET, host_out(D, torch).as_batch(), S.numpy())
        assert rc == 0
        assert_same_all(host_out(out, torch), want, N_DOCS, R)
        # the generated clocks saturate over thousands of docs (every rank's max
        # is 31); one rank-specific clock word per rank makes the summaries differ
        out.vv[3 * R + rank] = 1000 + rank
        want.vv[3 * R + rank] = 1000 + rank
        summ = torch.zeros(R, dtype=torch.int64, device=dev)
        eng.causal_context_async(out.vv, N_DOCS, R, summ)
        eng.sync()
        local = summ.cpu().numpy().view(np.uint64).tolist()
        oracle_local = oracle.causal_context(want.vv, N_DOCS, R).tolist()
        glob = cdist.u64_max_allreduce(dist, summ.cpu()).numpy().view(np.uint64).tolist()
        eng.close()
        dist.destroy_process_group()
        q.put((rank, local, oracle_local, glob, None))
    except Exception as e:  # reported to the parent, which fails the test
        q.put((rank, None, None, None, "%s: %s" % (type(e).__name__, e)))


def test_two_ranks_device_summaries_allreduce():
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
    errs = [r[4] for r in res if r[4]]
    assert not errs, errs
    assert all(p.exitcode == 0 for p in ps)
    for rank, local, oracle_local, _, _ in res:
        assert local == oracle_local, rank  # device summary == oracle max over the rank's docs
    want = [max(r[2][i] for r in res) for i in range(R)]  # oracle max over every doc of every rank
    for r in res:
        assert r[3] == want
    assert res[0][1] != res[1][1]  # the shards differ, so the all-reduce had work to do
