"""One-process-per-GPU data parallelism for the inference path.

Images are independent in eval (BN running stats, dropout off, per-image box
loops -- reference keypoint_model.py:143-199), so a global batch shards into
contiguous image ranges with no exchange in the data path.  The only
collectives are the result collation the serving path needs:
  * all_reduce(MAX) of the per-rank padded person count P (outputs are padded
    to the global max, reference :138,181-183);
  * all_gather of the fixed-size per-image keypoint / visibility slabs
    (340 B per person) -- tiny, latency-bound messages over RCCL/xGMI.
Heatmaps (213 KB per person) stay sharded unless asked for.
Works with any torch.distributed backend ("nccl" = RCCL on ROCm; "gloo" for
the CPU tests).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, stop) image range of ``rank``; the first total % world
    ranks take one extra image."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def global_max_persons(p_local: int, device, group=None) -> int:
    """all_reduce(MAX) of the per-rank person count.  Blocks on a host copy of
    the result; ``collate_outputs`` skips it whenever P is known up front."""
    t = torch.tensor([p_local], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def pad_persons(x: torch.Tensor, p: int) -> torch.Tensor:
    """Zero-pad dim 1 (persons) to ``p`` (reference pad_to_length semantics)."""
    if x.size(1) == p:
        return x
    pad = torch.zeros((x.size(0), p - x.size(1)) + tuple(x.shape[2:]), dtype=x.dtype, device=x.device)
    return torch.cat([x, pad], dim=1)


class PendingCollation:
    """The all_gathers of one collate_outputs(..., async_op=True) call in flight.
    ``wait()`` completes them (on RCCL: the caller's stream waits for the
    collective's stream, no host block) and returns the collated dict.  Until
    then the caller may enqueue more work -- the next batch's forward -- which
    then overlaps the collective instead of queueing behind it."""

    def __init__(self, items, group):
        self._items = items          # key -> (work, parts, counts, send buffer kept alive)
        self._group = group
        self._done = None

    def wait(self) -> Dict[str, torch.Tensor]:
        if self._done is None:
            res = {}
            for k, (work, parts, counts, _buf) in self._items.items():
                work.wait()
                res[k] = torch.cat([parts[r][: b - a] for r, (a, b) in enumerate(counts)], dim=0)
            self._done, self._items = res, None
        return self._done


def _gather_start(local: torch.Tensor, total: int, group, async_op: bool):
    world = dist.get_world_size(group)
    counts = [shard_range(total, world, r) for r in range(world)]
    mx = max(b - a for a, b in counts)
    if local.size(0) == mx:
        buf = local.contiguous()
    else:
        buf = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        buf[: local.size(0)] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    work = dist.all_gather(parts, buf, group=group, async_op=async_op)
    return work, parts, counts, buf


def gather_images(local: torch.Tensor, total: int, group=None) -> torch.Tensor:
    """all_gather a per-image tensor [n_local, ...] sharded by ``shard_range``
    into [total, ...] on every rank (uneven shards padded then trimmed)."""
    _work, parts, counts, _buf = _gather_start(local, total, group, False)
    return torch.cat([parts[r][: b - a] for r, (a, b) in enumerate(counts)], dim=0)


def collate_outputs(out: Dict[str, torch.Tensor], total: int, group=None,
                    keys: Sequence[str] = ("keypoints", "visibilities"),
                    max_persons: Optional[int] = None, async_op: bool = False):
    """Pad this rank's outputs to the global person count and all-gather ``keys``
    (add "heatmap" to collate the [n,P,17,56,56] heatmaps too: 213 KB per
    person).  ``max_persons``: the global padded person count when the caller
    knows it (a sharded [B,P,4] box tensor: P on every rank; the detector:
    max_persons) -- then no all_reduce and no host synchronisation happen.
    ``async_op``: return a PendingCollation whose ``wait()`` gives the dict
    (a serving loop collates batch k while batch k + 1 computes)."""
    p = max_persons
    if p is None:
        p = global_max_persons(out["keypoints"].size(1), out["keypoints"].device, group)
    if async_op:
        return PendingCollation({k: _gather_start(pad_persons(out[k], p), total, group, True) for k in keys}, group)
    res = {}
    for k in keys:
        res[k] = gather_images(pad_persons(out[k], p), total, group)
    return res


def sharded_forward(model, images: torch.Tensor, boxes: Optional[torch.Tensor], group=None,
                    keys: Sequence[str] = ("keypoints", "visibilities")) -> Dict[str, torch.Tensor]:
    """Run this rank's shard of a global batch and return the collated outputs
    of the whole batch on every rank.  ``boxes``: the global [B,P,4] box tensor
    (every rank's shard keeps the padded width P, so the collation needs no
    person-count exchange), or None for the person-detector branch (P =
    ``model.max_persons``)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    a, b = shard_range(images.size(0), world, rank)
    k = getattr(model, "num_keypoints", 17)
    p = boxes.size(1) if boxes is not None else int(getattr(model, "max_persons", 5))
    dev = images.device
    if b > a:
        out = model({"image": images[a:b], "bboxes": boxes[a:b]} if boxes is not None else images[a:b])
    elif p == 0:   # empty shard of a batch without boxes: the reference's all-empty shapes (:123-135)
        out = {"keypoints": torch.zeros(0, 1, k, 2, device=dev), "visibilities": torch.zeros(0, 1, k, device=dev),
               "heatmap": torch.zeros(0, 1, k, 56, 56, device=dev)}
    else:          # more ranks than images: contribute an empty shard
        out = {"keypoints": torch.zeros(0, p, 1, k, 2, device=dev),
               "visibilities": torch.zeros(0, p, 1, k, 3, device=dev),
               "heatmap": torch.zeros(0, p, k, 56, 56, device=dev)}
    # P = 0 (no box anywhere): every image returns one zero person
    return collate_outputs(out, images.size(0), group, keys, max_persons=max(p, 1))
