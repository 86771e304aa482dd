"""N>1 path on CPU: world_size-2 gloo processes exercise the image sharding,
the global person-count all_reduce and the result all_gather that bench.py /
dll.distributed use over RCCL on the GPU node."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeModel:
    """Deterministic per-image outputs; the person count depends on the shard
    (ranks see different P) to exercise the padding path."""
    num_keypoints = 17

    def __call__(self, batch):
        img, boxes = batch["image"], batch["bboxes"]
        n = img.size(0)
        p = boxes.size(1) - (1 if dist.get_rank() == 1 else 0)
        idx = img[:, 0, 0, 0]                       # carries the global image index
        k = idx.view(n, 1, 1, 1, 1).expand(n, p, 1, 17, 2) + torch.arange(p).view(1, p, 1, 1, 1) * 0.01
        v = torch.zeros(n, p, 1, 17, 3)
        v[..., 1] = 1.0
        return {"keypoints": k.contiguous(), "visibilities": v}


def _worker(rank, world, port, total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "keypoint-detection_amd"))
        from dll.distributed import sharded_forward, shard_range
        images = torch.zeros(total, 3, 8, 8)
        images[:, 0, 0, 0] = torch.arange(total, dtype=torch.float32)
        boxes = torch.rand(total, 3, 4)
        out = sharded_forward(FakeModel(), images, boxes)
        q.put((rank, out["keypoints"], out["visibilities"], [shard_range(total, world, r) for r in range(world)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total", [7, 8, 1])
def test_sharded_forward_gloo(total):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ranges = res[0][3]
    assert ranges[0][0] == 0 and ranges[-1][1] == total
    assert sum(b - a for a, b in ranges) == total
    for rank, k, v, _ in res:
        assert k.shape == (total, 3, 1, 17, 2) and v.shape == (total, 3, 1, 17, 3)
        for i in range(total):
            a1, b1 = ranges[1]
            on_rank1 = a1 <= i < b1
            np_ = 2 if on_rank1 else 3
            assert torch.allclose(k[i, :np_, 0, 0, 0], i + torch.arange(np_) * 0.01)
            assert not k[i, np_:].any() and not v[i, np_:].any()      # padded persons are zero
            assert torch.equal(v[i, :np_, 0, :, 1], torch.ones(np_, 17))
        # every rank holds the same collated result
        assert torch.equal(k, res[0][1]) and torch.equal(v, res[0][2])


def test_shard_range_properties():
    import sys
    from dll.distributed import shard_range
    for total in range(0, 40):
        for world in range(1, 9):
            rs = [shard_range(total, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1
