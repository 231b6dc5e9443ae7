"""N > 1 path on CPU: record sharding with world_size 2 over gloo.

Each rank takes a contiguous record range (workload.shard), digests it (here with the CPU oracle
standing in for the device call, which needs a GPU), and the shards are gathered.  The gathered
digests must equal the unsharded batch; the timing reduction is the bench's max-over-ranks.
No collective touches record data in the product path -- the all_gather here is the test's check.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from brb_framework_amd import workload


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, L, q):
    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r0, r1 = workload.shard(n, rank, world)
        data = workload.gen_records(workload.SEEDS[5], r0, r1 - r0, L)
        dig = oracle.md5_batch_fixed(data, L, r1 - r0)
        # variable-size shards: gather through a padded buffer + the true sizes
        size = torch.tensor([r1 - r0])
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, size)
        cap = int(max(s.item() for s in sizes))
        buf = torch.zeros((cap, 16), dtype=torch.uint8)
        buf[: r1 - r0] = torch.from_numpy(dig)
        bufs = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(bufs, buf)
        # the bench's timing reduction: max over ranks
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            full = np.concatenate([b[: int(s.item())].numpy() for b, s in zip(bufs, sizes)])
            q.put((full, float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [1000, 1025])
def test_sharded_digests_equal_unsharded(n):
    import oracle
    L = 1500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, L, q)) for r in range(2)]
    for p in procs:
        p.start()
    full, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = oracle.md5_batch_fixed(workload.gen_records(workload.SEEDS[5], 0, n, L), L, n)
    assert np.array_equal(full, want)
    assert tmax == 2.0


def test_shard_ranges_partition():
    for n in (0, 1, 7, 65536, 8 << 20):
        for world in (1, 2, 3, 4, 8):
            got = [workload.shard(n, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1
    # cfg5: 8 388 608 records over 8 GPUs = 1 048 576 each
    assert workload.shard(8 << 20, 7, 8) == (7 << 20, 8 << 20)
