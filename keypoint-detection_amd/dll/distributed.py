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

import math
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

    def __init__(self, packs, group):
        self._packs = packs          # [(keys, shapes, (work, out, counts, mx, widths, send buffer))]
        self._group = group
        self._done = None

    def wait(self) -> Dict[str, torch.Tensor]:
        if self._done is None:
            res = {}
            for keys, shapes, st in self._packs:
                st[0].wait()
                res.update(zip(keys, _unpack(st, shapes)))
            self._done, self._packs = res, None
        return self._done


def _gather_start(tensors: List[torch.Tensor], total: int, group, async_op: bool):
    """One all_gather_into_tensor of per-image tensors [n_local, ...] (same
    dtype and device), each flattened per image and laid side by side in one
    [n, W] send buffer: a single collective (and a single packing kernel) per
    call instead of one gather, its list copies and a concatenation per key."""
    world = dist.get_world_size(group)
    counts = [shard_range(total, world, r) for r in range(world)]
    mx = max(b - a for a, b in counts)
    n = tensors[0].size(0)
    flat = [t.reshape(n, math.prod(t.shape[1:])) for t in tensors]   # (explicit width: n may be 0)
    widths = [f.size(1) for f in flat]
    dt, dev = tensors[0].dtype, tensors[0].device
    if len(flat) == 1 and n == mx:
        buf = flat[0].contiguous()
    else:
        # a short shard (uneven split) is zero padded to mx images
        buf = (torch.empty if n == mx else torch.zeros)((mx, sum(widths)), dtype=dt, device=dev)
        if n and sum(widths):
            torch.cat(flat, dim=1, out=buf[:n])
    out = torch.empty((world * mx, sum(widths)), dtype=dt, device=dev)
    work = dist.all_gather_into_tensor(out, buf, group=group, async_op=async_op)
    return work, out, counts, mx, widths, buf


def _unpack(st, shapes) -> List[torch.Tensor]:
    """[total, ...] views of the gathered [world * mx, W] buffer, one per packed
    tensor (image-strided views: no copy when the shards are even)."""
    _work, out, counts, mx, widths, _buf = st
    if all(b - a == mx for a, b in counts):
        full = out
    else:
        full = torch.cat([out[r * mx: r * mx + (b - a)] for r, (a, b) in enumerate(counts)], dim=0)
    total, wsum = counts[-1][1], sum(widths)
    res, off = [], 0
    for w, shp in zip(widths, shapes):
        strides, acc = [], 1
        for d in reversed(shp):
            strides.insert(0, acc)
            acc *= d
        res.append(full.as_strided((total,) + tuple(shp), (wsum,) + tuple(strides), full.storage_offset() + off))
        off += w
    return res


def gather_images(local: torch.Tensor, total: int, group=None) -> torch.Tensor:
    """all_gather a per-image tensor [n_local, ...] sharded by ``shard_range``
    into [total, ...] on every rank (uneven shards padded then trimmed)."""
    return _unpack(_gather_start([local], total, group, False), [tuple(local.shape[1:])])[0]


def _packs(src: Dict[str, torch.Tensor], keys: Sequence[str], total: int, group, async_op: bool):
    """Keys grouped by (dtype, device) in order, one packed collective per group."""
    groups: Dict[tuple, List[str]] = {}
    for k in keys:
        groups.setdefault((src[k].dtype, src[k].device), []).append(k)
    return [(ks, [tuple(src[k].shape[1:]) for k in ks], _gather_start([src[k] for k in ks], total, group, async_op))
            for ks in groups.values()]


def collate_outputs(out: Dict[str, torch.Tensor], total: int, group=None,
                    keys: Sequence[str] = ("keypoints", "visibilities"),
                    max_persons: Optional[int] = None, async_op: bool = False):
    """Pad this rank's outputs to the global person count and all-gather ``keys``
    (add "heatmap" to collate the [n,P,17,56,56] heatmaps too: 213 KB per
    person).  ``max_persons``: the global padded person count when the caller
    knows it (a sharded [B,P,4] box tensor: P on every rank; the detector:
    max_persons) -- then no all_reduce and no host synchronisation happen.
    The keys travel packed side by side in one collective per dtype.
    ``async_op``: return a PendingCollation whose ``wait()`` gives the dict
    (a serving loop collates batch k while batch k + 1 computes)."""
    p = max_persons
    if p is None:
        p = global_max_persons(out["keypoints"].size(1), out["keypoints"].device, group)
    src = {k: pad_persons(out[k], p) for k in keys}
    packs = _packs(src, keys, total, group, async_op)
    if async_op:
        return PendingCollation(packs, group)
    res = {}
    for ks, shapes, st in packs:
        res.update(zip(ks, _unpack(st, shapes)))
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
