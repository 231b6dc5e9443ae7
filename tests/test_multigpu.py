"""N > 1 path: record sharding with world_size 2 (and 4 on the CPU) over gloo.

Each rank takes a contiguous record range (workload.shard, the same rule as the library's
BRB_BATCH_ALL_DEVICES split), digests it with the PRODUCT library, and the shards are gathered.  The
gathered digests must equal the oracle's digests of the unsharded batch; the timing reduction is the
bench's max-over-ranks.  No collective touches record data in the product path -- the all_gather here
is the test's check.
  * mode "compat" (CPU, runs here): every record through the library's compat surface
    (BRB_MD5Init / BRB_MD5Update / BRB_MD5Final, libbrb_crypto_gpu.so host code);
  * mode "gpu" (-m gpu): each rank's shard through BRB_MD5BatchFixed in device mode on its GPU
    (rank % visible devices: both ranks share the card on a one-GPU box).
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


def _digest_shard(mode, rank, data, L, m):
    import ctypes

    import brb_framework_amd as brb
    if mode == "gpu":
        dev = torch.device("cuda", rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        return brb.md5_batch_fixed(torch.from_numpy(data).to(dev), L, m).cpu().numpy()
    L_ = brb.lib()
    out = np.empty((m, 16), np.uint8)
    for i in range(m):
        c = brb.BRB_MD5_CTX()
        L_.BRB_MD5Init(ctypes.byref(c))
        L_.BRB_MD5Update(ctypes.byref(c), data[i * L:(i + 1) * L].tobytes(), L)
        L_.BRB_MD5Final(ctypes.byref(c))
        out[i] = np.frombuffer(bytes(c.digest), np.uint8)
    return out


def _worker(rank, world, port, n, L, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r0, r1 = workload.shard(n, rank, world)
        data = workload.gen_records(workload.SEEDS[5], r0, r1 - r0, L)
        dig = _digest_shard(mode, rank, data, L, r1 - r0)
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


def _run_sharded(n, mode, world=2):
    import oracle
    L = 1500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, L, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    full, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = oracle.md5_batch_fixed(workload.gen_records(workload.SEEDS[5], 0, n, L), L, n)
    assert np.array_equal(full, want)
    assert tmax == float(world)


@pytest.mark.parametrize("n,world", [(1000, 2), (1025, 2), (1027, 4)])
def test_sharded_compat_digests_equal_unsharded(n, world):
    _run_sharded(n, "compat", world)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [70_001])
def test_sharded_gpu_digests_equal_unsharded(n):
    _run_sharded(n, "gpu")


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
