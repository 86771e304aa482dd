#!/usr/bin/env python3
"""Benchmark: images/sec of MultiPersonKeypointModel.forward (eval, given boxes)
on the BASELINE.json headline config C2 -- batch 64 per GPU, synthetic
256x192x3 images, 1 person box per image, 17 COCO keypoints, heatmap head +
soft-argmax decode -- through the native HIP path.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One process per GPU; images shard across ranks (weak scaling, B per rank) and
each step all-gathers the per-image keypoints/visibilities to every rank over
RCCL (result collation), pipelined one step deep: step k's all_gather runs
under step k + 1's forward, the last one completes inside the timed region.
With N > 1 the labelled `configs.C4` (the C3 pipeline per rank) and
`configs.C5` objects do the same for the full pipeline.  Rank 0 prints one JSON line with the
whole-job rate, the dominant kernel's roofline fraction (HIP events on the
launch stream, inside the timed region) and the CPU-oracle baseline timed on
this host (N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for _p in (str(ROOT), str(ROOT / "keypoint-detection_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

PEAK_TFLOPS = {"fp32": 157.3, "bf16": 2500.0}   # MI355X dense MFMA peaks (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def conv_flops(cin, cout, k, h, w, groups=1):
    return 2.0 * cout * (cin // groups) * k * k * h * w


# torchvision mobilenet_v3_small features.1-11 rows (in, k, exp, out, SE, act,
# stride) -- the architecture table, used here only to count FLOPs
BNECK = ((16, 3, 16, 16, True, "RE", 2), (16, 3, 72, 24, False, "RE", 2), (24, 3, 88, 24, False, "RE", 1),
         (24, 5, 96, 40, True, "HS", 2), (40, 5, 240, 40, True, "HS", 1), (40, 5, 240, 40, True, "HS", 1),
         (40, 5, 120, 48, True, "HS", 1), (48, 5, 144, 48, True, "HS", 1), (48, 5, 288, 96, True, "HS", 2),
         (96, 5, 576, 96, True, "HS", 1), (96, 5, 576, 96, True, "HS", 1))


def _make_divisible(v, d=8):
    n = max(d, int(v + d / 2) // d * d)
    return n + d if n < 0.9 * v else n


def flops_per_image(H, W, P, in_ch=3):
    """Algorithmic FLOPs (2*MAC of conv/linear, BN folded, dead FPN levels 1-3
    excluded) -- SURVEY.md §8(d)."""
    h, w = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    f = conv_flops(in_ch, 16, 3, h, w)
    sizes = [(h, w)]
    for cin, k, exp, cout, se, _a, s in BNECK:
        if exp != cin:
            f += conv_flops(cin, exp, 1, h, w)
        ho, wo = (h + 2 * ((k - 1) // 2) - k) // s + 1, (w + 2 * ((k - 1) // 2) - k) // s + 1
        f += conv_flops(exp, exp, k, ho, wo, groups=exp)
        if se:
            sq = _make_divisible(exp // 4, 8)
            f += 2.0 * (exp * sq * 2)
        f += conv_flops(exp, cout, 1, ho, wo)
        h, w = ho, wo
        sizes.append((h, w))
    f += conv_flops(96, 576, 1, h, w)
    taps = [sizes[0], sizes[3], sizes[8], sizes[11]]
    for cin, (th, tw) in zip((16, 24, 48, 576), taps):
        f += conv_flops(cin, 128, 1, th, tw)
    fpn0 = conv_flops(128, 128, 3, *sizes[0])
    f += fpn0 + 2.0 * (128 * 8 * 2) * 2
    hm_convs = [conv_flops(64, 256, 3, 56, 56), conv_flops(256, 256, 3, 56, 56), conv_flops(256, 64, 3, 56, 56)]
    head = sum(hm_convs) + conv_flops(64, 17, 1, 56, 56) + conv_flops(2, 1, 7, 56, 56) + 2.0 * (64 * 4 * 2) * 2
    return {"total": f + P * head, "fpn0": fpn0, "hm_conv1": hm_convs[0] * P, "hm_conv2": hm_convs[1] * P,
            "hm_conv3": hm_convs[2] * P}


def kh_flops_per_roi(c=128, fine=64, reg=32, vis=32, h=56, w=56, attention=True):
    """KEYPOINT_HEAD algorithmic flops per ROI (keypoint_head.py:9-90): 2*MAC
    of its convs and linears at the ROI resolution (BN folded); attention=False
    leaves out the spatial attention's 1x1 convs (fused into the ROI align
    kernel, roi_kh_kernel, so timed in the roi_align stage)."""
    hw = h * w
    f = 2.0 * hw * (c * (c // 2) + (c // 2)) if attention else 0.0   # spatial attention 1x1 C->C/2->1
    f += 2.0 * hw * (c * fine * 9 + (c * fine if c != fine else 0))  # ResidualBlock(C->64) (+ downsample)
    f += 2.0 * hw * (fine * reg * 9 + (fine * reg if fine != reg else 0))
    f += 2.0 * hw * reg * (reg // 2) * 9                               # 3x3 32->16
    f += 2.0 * ((reg // 2) * (h // 4) * (w // 4) * 256 + 256 * 34)    # regression linears
    f += 2.0 * hw * c * vis * 9 + 2.0 * (vis * 16 * 128 + 128 * 51)   # visibility branch
    return f


def config_flops(H, W, P, detect):
    """Per-image algorithmic flops of a C3 / C5 forward: backbone
    + FPN level 0 + P x (heatmap head + KEYPOINT_HEAD) (+ the detector's 1x1
    heads on the 56x56-pooled 128-channel level 0).  P may be fractional (the
    mean detected persons per image)."""
    fl = dict(flops_per_image(H, W, P))
    kh = kh_flops_per_roi()
    fl["keypoint_head"] = P * kh
    fl["keypoint_head_convs"] = P * kh_flops_per_roi(attention=False)
    fl["total"] += P * kh + (2.0 * 3136 * 128 * 45 if detect else 0.0)
    return fl


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50,
                    help="untimed forwards first: the GPU clock ramps over the first ~30 (hm conv 2 0.57 -> 0.51 ms)")
    ap.add_argument("--batch", type=int, default=64, help="images per GPU per step")
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=192)
    ap.add_argument("--persons", type=int, default=1)
    ap.add_argument("--precision", default="split", choices=["fp32", "split", "mixed"],
                    help="split = fp32-accurate (the reference's precision); mixed = bf16 heatmap convs")
    ap.add_argument("--secondary", default="mixed", help="second, labelled precision line at N=1 ('' = none)")
    ap.add_argument("--no-exact-check", dest="exact_check", action="store_false",
                    help="skip the exact-product fp32 cross-check object (N=1)")
    ap.add_argument("--cpu-sample", type=int, default=64, help="images in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--streams", type=int, default=1,
                    help="sub-batch streams inside one forward (kpd_plan_set_streams); 2 overlaps the sub-batches "
                         "(~4%% more images/s) but then every kernel shares the GPU and its launch time no longer "
                         "describes the kernel")
    ap.add_argument("--alt-streams", type=int, default=2,
                    help="N=1: also time the same workload at this many sub-batch streams (labelled "
                         "'alt_streams'; 0 = skip); the headline stays single-stream so the roofline's launch "
                         "times describe the kernel alone")
    ap.add_argument("--pmc-json", default=str(ROOT / "profiles" / "r06" / "pmc.json"),
                    help="per-launch HBM traffic of the dominant kernel from a rocprofv3 --pmc run (entries are "
                         "stamped with the hash of the kernel sources they were measured on)")
    ap.add_argument("--configs", default="auto",
                    help="labelled BASELINE config objects after the C2 headline: 'auto' = C1,C3,C5 at N=1 and "
                         "C4,C5 at N>1 (C4 = the C3 pipeline per rank with RCCL collation); a comma list; 'none'")
    ap.add_argument("--only", default=None, choices=sorted(PIPELINES) + ["C1"],
                    help="run only this config object (profiling passes)")
    ap.add_argument("--c3-only", dest="only", action="store_const", const="C3", help="= --only C3")
    ap.add_argument("--cfg-batch", type=int, default=0, help="images per rank of the config objects (0 = theirs)")
    ap.add_argument("--cfg-cpu-sample", type=int, default=8, help="images in the config objects' CPU-baseline sample")
    ap.add_argument("--force-dist", action="store_true",
                    help="test hook: initialise the process group (RCCL) and run the N-rank code paths -- "
                         "collation, barriers, max-over-ranks timing -- even at one rank")
    ap.add_argument("--cpu-standin", action="store_true",
                    help="test mode: no GPU; gloo ranks on the CPU run a stand-in forward through the same "
                         "launcher, barrier, timing and collation code (tests/test_bench_launch.py)")
    return ap.parse_args(argv)


def host_cpu_info():
    """CPU model, machine core counts and the CPU share this process may use
    (cgroup v2 cpu.max quota / affinity), for the baseline's `cores`."""
    info = {"model": None, "physical_cores": None, "logical_cpus": os.cpu_count(), "cgroup_cpus": None}
    try:
        phys, model = set(), None
        with open("/proc/cpuinfo") as fh:
            pid = cid = None
            for line in fh:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and model is None:
                    model = v
                elif k == "physical id":
                    pid = v
                elif k == "core id":
                    cid = v
                elif not k and pid is not None:
                    phys.add((pid, cid))
                    pid = cid = None
        info["model"], info["physical_cores"] = model, len(phys) or None
    except OSError:
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            info["cgroup_cpus"] = int(q) // int(per)
    except (OSError, ValueError):
        pass
    avail = [len(os.sched_getaffinity(0))]
    if info["cgroup_cpus"]:
        avail.append(info["cgroup_cpus"])
    if info["physical_cores"]:
        avail.append(info["physical_cores"])
    info["threads"] = max(1, min(avail))
    return info


def cpu_baseline(sd, img, boxes, threads, warmups=3, runs=5, max_seconds=40.0, fwd=None):
    """The oracle (a plain-torch restatement of the reference forward with its
    per-box loop, golden-pinned) timed on this host: `warmups` untimed runs,
    then the median of `runs` timed runs of the whole sample (more runs if
    they fit in max_seconds, never fewer than 5).  `fwd` replaces the default
    given-box forward (C3: dual head + detector glue)."""
    from oracle import kpd_oracle as O
    torch.set_num_threads(threads)
    batch = {"image": img, "bboxes": boxes}
    if fwd is None:
        def fwd():
            return O.forward(sd, batch)
    t0 = time.perf_counter()
    out = fwd()                       # first warmup: also the parity outputs
    once = time.perf_counter() - t0
    warmups = max(1, min(warmups, int(max_seconds / 3 / max(once, 1e-3))))
    for _ in range(warmups - 1):
        fwd()
    runs = max(5, min(runs, int(max_seconds / max(once, 1e-3))))
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        fwd()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    med = ts[len(ts) // 2]
    return out, img.shape[0] / med, {"warmups": warmups, "runs": runs, "median_s": round(med, 4),
                                     "min_s": round(ts[0], 4), "max_s": round(ts[-1], 4)}


def _cuda_sync():
    torch.cuda.synchronize()


def run_steps(steps, warmup, step_fn, dist, sync=_cuda_sync, finish=None):
    """W untimed + K timed steps: barrier + synchronize, clock, the steps,
    synchronize, clock, barrier; seconds (the max over ranks is the job time).
    finish(): completes work a step leaves in flight (the last step's result
    collation), inside the timed region, before the closing synchronize."""
    import torch.distributed as tdist
    with torch.no_grad():
        for _ in range(warmup):
            step_fn()
        if finish:
            finish()
        sync()
        if dist:
            tdist.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = step_fn()
        if finish:
            finish()
        sync()
        # every rank's time from the common start barrier to its own last
        # synchronize; the job time is the max over ranks (gather_elapsed).
        # The closing barrier follows the clock read: a RCCL barrier costs
        # ~1.8 ms at its call, which is synchronisation, not the K steps.
        el = time.perf_counter() - t0
        if dist:
            tdist.barrier()
        return el, out


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`--gpus N` (N > 1) without a launcher: start N ranks (one per GPU) through
    torch.distributed.run as a child process and return its exit code.  This
    process never touches the GPU (no HIP call before or after), and rank 0 of
    the children prints the JSON line on the inherited stdout."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC only on this host driver (RCCL)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(Path(__file__).resolve())] + argv
    return subprocess.run(cmd, env=env).returncode


class StandinModel:
    """--cpu-standin: a cheap deterministic forward with the drop-in's output
    contract ([n,P,1,17,2] keypoints, [n,P,1,17,3] one-hot visibilities,
    [n,P,17,56,56] heatmaps, the dual head's kh_* outputs; without boxes the
    detector branch's P = max_persons, box list and box_scores), so the
    launcher / timing / collation code runs without a GPU.  keypoints[..., 0]
    carry (offset + local image index) / 1e4, so a collated copy shows where
    every rank's slab landed.  It is not the model and never produces a bench
    number."""
    num_keypoints = 17

    def __init__(self, offset=0, max_persons=5):
        self.offset, self.max_persons = offset, max_persons

    def __call__(self, batch):
        img = batch["image"] if isinstance(batch, dict) else batch
        n = img.size(0)
        if isinstance(batch, dict) and "bboxes" in batch:
            boxes = batch["bboxes"]
        else:
            g = torch.Generator().manual_seed(self.offset)
            boxes = torch.rand(n, self.max_persons, 4, generator=g)
        p = boxes.size(1)
        m = img.mean(dim=(1, 2, 3))
        k = (boxes[..., :2].unsqueeze(2) + 0.01 * m.view(n, 1, 1, 1)).expand(n, p, 17, 2).clamp(0, 1).clone()
        k[..., 0] = ((self.offset + torch.arange(n, dtype=torch.float32)) / 1e4).view(n, 1, 1)
        v = torch.zeros(n, p, 17, 3)
        v[..., 2] = 1.0
        out = {"keypoints": k.unsqueeze(2).contiguous(), "visibilities": v.unsqueeze(2),
               "heatmap": torch.zeros(n, p, 17, 56, 56), "kh_keypoints": k.unsqueeze(2) * 0.5,
               "kh_visibilities": v.unsqueeze(2) * 0.5, "boxes": [boxes[i] for i in range(n)]}
        if not (isinstance(batch, dict) and "bboxes" in batch):
            out["box_scores"] = boxes[..., 0].clone()
        return out


class Collator:
    """Result collation pipelined one step deep: step k starts the all_gathers
    of its outputs (async) after waiting for step k - 1's, so each step's
    collective runs under the next step's forward instead of in series with it
    (dll.distributed.collate_outputs(..., async_op=True)); finish() completes
    the last one (run_steps calls it inside the timed region).  The collated
    tensors of the latest completed step land in ``into``."""

    def __init__(self, total, keys, max_persons, into):
        self.total, self.keys, self.p, self.into, self.pending = total, keys, max_persons, into, None

    def start(self, out):
        from dll.distributed import collate_outputs
        src = {k: out[k] for k in self.keys}
        self.finish()
        self.pending = collate_outputs(src, self.total, keys=self.keys, max_persons=self.p, async_op=True)

    def finish(self):
        if self.pending is not None:
            self.into.update(self.pending.wait())
            self.pending = None


def main_standin(a, world, rank, dist):
    """The N-rank code path of main() with gloo on the CPU and StandinModel."""
    import torch.distributed as tdist
    from dll.distributed import collate_outputs
    from dll.models.synthetic import synthetic_boxes, synthetic_images
    torch.set_num_threads(1)
    B, P = a.batch, a.persons
    img = synthetic_images(B, 3, a.height, a.width, seed=1234 + 7919 * rank)
    boxes = synthetic_boxes(B, P, seed=1235 + 7919 * rank)
    batch = {"image": img, "bboxes": boxes}
    model = StandinModel()
    gather = dist and not a.no_gather
    coll = {}
    pend = Collator(B * world, ("keypoints", "visibilities"), P, coll)

    def step():
        out = model(batch)
        if gather:
            pend.start(out)
        return out

    el, _ = run_steps(a.steps, a.warmup, step, dist, sync=lambda: None, finish=pend.finish)
    per_rank = gather_elapsed(el, world, dist, torch.device("cpu"))
    el = max(per_rank)
    line = {"metric": "cpu-standin (launcher test; not a measurement)", "value": round(B * world * a.steps / el, 2),
            "unit": "images/s", "n_gpus": world, "world": world, "backend": "gloo" if dist else None,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 4),
            "rank_ms_per_step": [round(t / a.steps * 1e3, 4) for t in per_rank],
            "rccl_ranks": rank_census(dist, torch.device("cpu")),
            "collated": {k: list(v.shape) for k, v in coll.items()}}
    if gather:   # every rank's slab landed at its shard's offset
        from dll.distributed import shard_range
        line["collated_ok"] = collation_check(model(batch), coll, ("keypoints", "visibilities"), P, world, rank,
                                              dist, torch.device("cpu"))
        line["collated_index_ok"] = bool(all(
            torch.equal(coll["visibilities"][s:e, :, 0, :, 2], torch.ones(e - s, P, 17))
            for s, e in (shard_range(B * world, world, r) for r in range(world))))
    cfgs = {}
    for name in config_names(a, world, standin=True):
        cfgs[name] = run_pipeline(name, a, torch.device("cpu"), None, world, rank, dist, cpu=False, standin=True)
    if cfgs:
        line["configs"] = cfgs
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


def rank_census(dist, dev):
    """Ranks in the process group, counted by an all_reduce(SUM) of ones over
    the data-path backend (RCCL on the GPU ranks, gloo for the stand-in): a
    self-check that every rank took part in the collectives; None without a
    process group."""
    if not dist:
        return None
    import torch.distributed as tdist
    t = torch.ones(1, device=dev, dtype=torch.int32)
    tdist.all_reduce(t)
    return int(t.item())


def gather_elapsed(el, world, dist, dev):
    """Every rank's elapsed seconds (all_gather; the job time is their max)."""
    t = torch.tensor([el], device=dev, dtype=torch.float64)
    if not dist:
        return [el]
    import torch.distributed as tdist
    parts = [torch.empty_like(t) for _ in range(world)]
    tdist.all_gather(parts, t)
    return [float(x.item()) for x in parts]


def stage_pass(m, plan, batch, iters):
    """Per-stage HIP-event means (events on each sub-batch's launch stream) of
    `iters` forwards in the run's own configuration (same sub-batch streams,
    so every kernel launch has the shape the timed region launches)."""
    from dll import _native
    with torch.no_grad():
        torch.cuda.synchronize()
        plan.timing(True)
        for _ in range(iters):
            m(batch)
        torch.cuda.synchronize()
        plan.timing(False)
    st = {}
    for s in _native.STAGES:
        ms, n = plan.timing_query(s)
        if n:
            st[s] = (ms / n, n)
    return st


def roofline(precision, stages, fl, B, H, W, pmc, dom=None, tag=None):
    """Roofline of the dominant kernel (the longest single-kernel MFMA stage).
    achieved = ALGORITHMIC flops per launch / mean launch time;
    peak = dense MFMA peak of the dtype the kernel issues (f16/bf16 2.5 PF,
    f32 157.3 TF).  The MFMA work actually issued (split products, padded
    border rows, FPN level 0 by linearity) is reported beside it."""
    hf, wf = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    h1, w1 = hf, wf
    for _cin, k, _e, _co, _se, _a, st in BNECK[:3]:
        pd = (k - 1) // 2
        h1, w1 = (h1 + 2 * pd - k) // st + 1, (w1 + 2 * pd - k) // st + 1
    split_fpn = precision in ("split", "mixed") and hf == 4 * h1 and wf == 4 * w1
    pad = 57 * 57 / (56 * 56)    # hmconv computes every position of the 57x57 layout (borders discarded)
    kern = {}
    if split_fpn:
        ex = 3 * 2.0 * hf * wf * (5 * 32 * 128 + 36 * 128 * 128 / 16) * B
        kern["fpn0"] = (fl["fpn0"] * B, PEAK_TFLOPS["bf16"], ex, "fpn0x_kernel",
                        "FPN level-0 conv3x3 128->128 by linearity (composite 16-ch 3x3 on the stem tap + per-"
                        "position-class lateral-1 tap groups), fp32-accurate: 3 f16 products per MAC on "
                        "v_mfma_f32_16x16x32_f16")
    else:
        kern["fpn0"] = (fl["fpn0"] * B, PEAK_TFLOPS["fp32"], fl["fpn0"] * B, "conv_mfma_kernel",
                        "FPN level-0 conv3x3 on v_mfma_f32_16x16x4_f32")
    for s in ("hm_conv1", "hm_conv2", "hm_conv3"):
        f = fl[s] * B
        if precision == "split":
            kern[s] = (f, PEAK_TFLOPS["bf16"], 3 * f * pad, "hmconv_kernel<SPLIT>",
                       f"{s} conv3x3 on the zero-bordered hmconv layout, fp32-accurate: 3 f16 products per MAC on "
                       "v_mfma_f32_16x16x32_f16")
        elif precision == "mixed":
            kern[s] = (f, PEAK_TFLOPS["bf16"], f * pad, "hmconv_kernel",
                       f"{s} conv3x3 on the zero-bordered hmconv layout, bf16 operands on v_mfma_f32_16x16x32_bf16")
        else:
            kern[s] = (f, PEAK_TFLOPS["fp32"], f, "conv_mfma_kernel", f"{s} conv3x3 on v_mfma_f32_16x16x4_f32")
    if precision == "split":
        kern["hm_conv2"] += ("one stage = two launches: complete rounds of 224-row tiles "
                             "(hmconv_kernel<256, 2, 0, 224, true, 256>) + the remaining rows as 160-row tiles "
                             "(hmconv_kernel<256, 2, 0, 160, true, 256>; 192-row when 160 would need a second "
                             "round); their rocprofv3 averages sum to avg_ms",)
    if precision in ("split", "mixed"):
        kern["hm_conv3"] += ("one stage = two launches: complete rounds of 256-row tiles + the remaining rows as "
                             "128-row tiles; their rocprofv3 averages sum to avg_ms",)
    cand = [s for s in kern if s in stages]
    if not cand:
        return None
    if dom is None:
        dom = max(cand, key=lambda k: stages[k])
    flop, peak, exflop, kname, desc = kern[dom][:5]
    note = kern[dom][5] if len(kern[dom]) > 5 else None
    t = stages[dom] * 1e-3
    ach, exa = flop / t / 1e12, exflop / t / 1e12
    r = {"bound": "mfma", "kernel": kname, "desc": desc, "stage": dom, "achieved": round(ach, 2), "peak": peak,
         "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": None,
         "flop_per_launch": flop, "avg_ms": round(stages[dom], 4),
         "executed_flop_per_launch": exflop, "executed_achieved": round(exa, 2),
         "executed_frac": round(exa / peak, 4)}
    if note:
        r["launches_note"] = note
    if exflop > 2.5 * flop:   # 3-product split: each fp32 MAC costs 3 MFMA products
        r["split_ceiling_frac"] = round(ach / (peak / 3.0), 4)
    # PMC entries: "<stage>:<precision>" for the headline C2, "<stage>:<precision>@<config>" otherwise
    e = pmc.get(f"{dom}:{precision}" + (f"@{tag}" if tag else "")) if pmc else None
    if e:
        r["traffic"] = e.get("hbm_bytes_per_launch")
        r["traffic_unit"] = "HBM bytes/launch: rocprofv3 --pmc, 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950)"
        if e.get("SQ_VALU_MFMA_BUSY_CYCLES") and e.get("GRBM_GUI_ACTIVE"):
            # MFMA-busy cycles summed over the 1024 SIMDs / (GUI-active cycles per XCD)
            r["mfma_busy_frac"] = round(e["SQ_VALU_MFMA_BUSY_CYCLES"] / (128.0 * e["GRBM_GUI_ACTIVE"]), 4)
        r["pmc_source"] = e.get("source")
        cur = kernel_src_hash()
        r["pmc_src_hash"] = e.get("src_hash")
        # the counters were measured on these kernel sources: false = stale (kernel changed since)
        r["pmc_current"] = e.get("src_hash") == cur
    return r


# BASELINE.json configs beyond the C2 headline, as labelled objects of the
# line (per-rank batch: B images on every rank, global B x N)
PIPELINES = {
    "C3": dict(B=256, H=256, W=192, P=None, max_persons=5, img_seed=4321,
               desc="C3: batch {B}, {H}x{W}x3, no boxes: person detector (pooled 1x1 heads, anchor decode, conf 0.3, "
                    "NMS 0.3, max 5) + heatmap head + soft-argmax + KEYPOINT_HEAD per detected ROI"),
    "C4": dict(B=256, H=256, W=192, P=None, max_persons=5, img_seed=4321,
               desc="C4: the C3 pipeline sharded {B} images/rank over {N} GPUs (global batch {G}; 2048 at 8 GPUs), "
                    "RCCL all_gather of keypoints / visibilities / KEYPOINT_HEAD outputs / boxes / box scores every "
                    "step"),
    "C5": dict(B=256, H=384, W=288, P=5, max_persons=5, img_seed=1234, box_seed=1235,
               desc="C5: {B} images/rank ({N} GPU(s), global batch {G}; 2048 at 8 GPUs), {H}x{W}x3, 5 given boxes/img, "
                    "heatmap head + soft-argmax + KEYPOINT_HEAD per box"
                    "{gather}"),
}
# outputs collated over ranks (dll.distributed.collate_outputs) for each config
COLLATE_KEYS = {"C3": ("keypoints", "visibilities", "kh_keypoints", "kh_visibilities", "box_scores", "boxes"),
                "C5": ("keypoints", "visibilities", "kh_keypoints", "kh_visibilities")}
COLLATE_KEYS["C4"] = COLLATE_KEYS["C3"]


def slab_sums(t, total, world):
    """float64 sum of each rank's [start, stop) image slab of a collated tensor."""
    from dll.distributed import shard_range
    return torch.stack([t[s:e].double().sum() for s, e in (shard_range(total, world, r) for r in range(world))])


def collation_check(local, coll, keys, P, world, rank, dist, dev):
    """Every rank's slab landed at its shard's offset in every rank's collated
    copy: each rank's local (padded) outputs are summed per key in float64,
    all_gathered, and compared with the sums of the collated slabs; the
    verdict is AND-reduced over ranks (1 = all ranks agree)."""
    import torch.distributed as tdist
    from dll.distributed import pad_persons
    mine = torch.stack([pad_persons(local[k], P).double().sum() for k in keys]).to(dev)
    allv = [torch.empty_like(mine) for _ in range(world)]
    tdist.all_gather(allv, mine)
    total = coll[keys[0]].size(0)
    ok = all(torch.equal(slab_sums(coll[k], total, world).to(dev), torch.stack([a[i] for a in allv]))
             for i, k in enumerate(keys))
    flag = torch.tensor([1 if ok else 0], device=dev, dtype=torch.int32)
    tdist.all_reduce(flag, op=tdist.ReduceOp.MIN)
    return bool(flag.item())


def run_pipeline(name, a, dev, pmc, world=1, rank=0, dist=False, cpu=True, standin=False):
    """One BASELINE pipeline config on this rank's GPU (C3 / C4 / C5; see
    PIPELINES), the dual head on every ROI.  Timed like the headline: W
    warm-ups, K forwards between barriers (max over ranks; at N > 1 each step
    also all-gathers the collated outputs over RCCL), HIP events around the
    dominant MFMA stage only; its roofline traffic from the PMC entry of the
    same per-GPU workload.  N = 1, rank 0: CPU baseline = the oracle's forward
    of the same config on the first --cfg-cpu-sample images (3 warm-ups +
    median of 5) and parity against it; C3 also at --alt-streams sub-batch
    streams (throughput only).  standin: gloo ranks on the CPU with
    StandinModel (launcher / collation test, no measurement)."""
    from dll.models.synthetic import synthetic_boxes, synthetic_images, synthetic_state_dict
    c = PIPELINES[name]
    B = a.cfg_batch or c["B"]
    H, W, P, Pk = c["H"], c["W"], c["P"], c["max_persons"]
    detect = P is None
    gather = dist and not a.no_gather
    keys = COLLATE_KEYS[name]
    img_cpu = synthetic_images(B, 3, H, W, seed=c["img_seed"] + 7919 * rank)
    box_cpu = None if detect else synthetic_boxes(B, P, seed=c["box_seed"] + 7919 * rank)
    if standin:
        m = StandinModel(offset=rank * B, max_persons=Pk)
        img = img_cpu
        sync = (lambda: None)
    else:
        from dll.configs import KeypointHeadConfig, ModelConfig, TrainingConfig
        from dll.models import MultiPersonKeypointModel
        m = MultiPersonKeypointModel(ModelConfig(keypoint_head=KeypointHeadConfig(height=56, width=56)),
                                     TrainingConfig(), precision=a.precision, dual_head=True, max_persons=Pk,
                                     streams=1)
        m.load_state_dict(synthetic_state_dict(m.state_dict(), seed=0))
        m = m.to(dev).eval()
        img = img_cpu.to(dev)
        sync = _cuda_sync
    batch = img if detect else {"image": img, "bboxes": box_cpu.to(img.device)}
    coll = {}
    pend = Collator(B * world, keys, Pk, coll)

    def step():
        out = m(batch)
        if gather:   # result collation over RCCL (P = max_persons on every rank: no host sync), one step deep
            if "boxes" in keys:
                out["boxes_t"] = torch.stack(out["boxes"])
            pend.start({k: out["boxes_t" if k == "boxes" else k] for k in keys})
        return out

    gN = B * world
    res = {"workload": c["desc"].format(B=B, H=H, W=W, N=world, G=gN,
                                        gather=", RCCL all_gather of keypoints / visibilities / KEYPOINT_HEAD "
                                               "outputs every step" if gather else ""),
           "images_per_rank": B, "global_batch": gN, "n_gpus": world, "precision": a.precision}
    if standin:
        el, out = run_steps(a.steps, a.warmup, step, dist, sync=sync, finish=pend.finish)
        stages, dom = {}, None
    else:
        from dll import _native  # noqa: F401
        plan = m.native_plan(dev)
        with torch.no_grad():
            for _ in range(a.warmup):
                step()
            pend.finish()
        bd = stage_pass(m, plan, batch, 1)
        launches = {k: v[1] for k, v in bd.items()}
        mfma_stages = ("fpn0", "hm_conv1", "hm_conv2", "hm_conv3")
        dom = max((k for k in bd if k in mfma_stages), key=lambda k: bd[k][0])
        plan.timing(True, stage=dom)
        el, out = run_steps(a.steps, 0, step, dist, finish=pend.finish)
        plan.timing(False)
        dms, dn = plan.timing_query(dom)
        stages = {k: v[0] for k, v in bd.items()}
        if dn:
            stages[dom] = dms / dn
    per_rank = gather_elapsed(el, world, dist, dev)
    el = max(per_rank)
    res.update({"value": round(gN * a.steps / el, 2), "unit": "images/s", "ms_per_step": round(el / a.steps * 1e3, 4),
                "rank_ms_per_step": [round(t / a.steps * 1e3, 4) for t in per_rank],
                "steps": a.steps, "warmup": a.warmup, "streams_per_gpu": 1, "scaling": "weak",
                "rccl_ranks": rank_census(dist, dev)})
    if gather:
        res["collated"] = {k: list(v.shape) for k, v in coll.items()}
        res["collated_ok"] = collation_check(out if "boxes" not in keys else dict(out, boxes=out["boxes_t"]),
                                             coll, keys, Pk, world, rank, dist, dev)
        res["collective"] = ("all_gather over " + ("gloo (CPU stand-in)" if standin else "RCCL (nccl backend)") +
                             f" of {', '.join(keys)} per step, padded to {Pk} persons")
    if standin:
        if gather:   # the stand-in encodes the global image index: every slab at its offset
            idx = torch.arange(gN, dtype=torch.float32)
            res["collated_index_ok"] = bool(torch.equal(coll["keypoints"][:, :, 0, :, 0],
                                                        (idx / 1e4).view(gN, 1, 1).expand(gN, Pk, 17)))
        return res
    rois = int((out["box_scores"] > 0).sum()) if detect else int((box_cpu.abs().sum(-1) > 0).sum())
    P_eff = rois / B                     # persons per image the heads ran on
    nl = max(1, launches[dom])           # launches of a stage per forward (one per pass)
    fl = config_flops(H, W, P_eff, detect)
    tag = "C3" if name == "C4" else name   # C4's per-GPU work is C3's: its single-GPU PMC entry
    roof = roofline(a.precision, stages, fl, B / nl, H, W, pmc, dom, tag=tag)
    roof["launches_timed"] = dn
    roof["images_per_launch"] = B / nl
    roof["rois_per_launch"] = rois / nl
    roof["timing"] = "HIP events around every launch of this stage inside the timed region (single stream)"
    if name == "C4":
        roof["pmc_note"] = "traffic / busy: the single-GPU C3 PMC entry (C4's per-rank workload is C3's)"
    res.update({"rois": rois, "persons_per_image": round(P_eff, 3), "gflop_per_image": round(fl["total"] / 1e9, 3),
                "achieved_tflops_total": round(fl["total"] * gN * a.steps / el / 1e12, 2), "roofline": roof,
                "stages_ms": {k: round(v, 4) for k, v in stages.items()}, "stage_launches_per_forward": launches})
    if "keypoint_head" in stages:
        # the keypoint_head stage runs the KEYPOINT_HEAD convs, pools and linears; its spatial attention
        # (1x1 128->64->1) is fused into the roi_align stage's kernel (roi_kh_kernel) in split precision
        fused = a.precision != "fp32"
        kf = fl["keypoint_head_convs"] if fused else fl["keypoint_head"]
        res["keypoint_head_tflops"] = round(kf * B / nl / (stages["keypoint_head"] * 1e-3) / 1e12, 2)
        res["keypoint_head_note"] = ("algorithmic KEYPOINT_HEAD flops of the keypoint_head stage / its time"
                                     + ("; the spatial attention's 1x1 convs run fused in the roi_align stage"
                                        if fused else ""))
    if name == "C3" and world == 1 and a.alt_streams and a.alt_streams != 1:
        m.streams = a.alt_streams
        el2, out2 = run_steps(a.steps, a.warmup, step, False)
        m.streams = 1
        res["alt_streams"] = {"streams_per_gpu": a.alt_streams, "value": round(B * a.steps / el2, 2),
                              "ms_per_step": round(el2 / a.steps * 1e3, 4),
                              "outputs_identical": all(torch.equal(out[k], out2[k]) for k in
                                                       ("keypoints", "visibilities", "kh_keypoints",
                                                        "box_scores"))}
    if cpu and world == 1 and rank == 0 and a.cfg_cpu_sample > 0:
        from oracle import kpd_oracle as O
        ci = host_cpu_info()
        S = min(a.cfg_cpu_sample, B)
        sdc = {k: v.cpu() for k, v in m.state_dict().items()}
        xs = img_cpu[:S]
        bs = None if detect else box_cpu[:S]

        def fwd():
            if detect:
                return O.forward(sdc, {"image": xs}, dual_head=True,
                                 detect=dict(conf_threshold=0.3, iou_threshold=0.3, max_persons=Pk))
            return O.forward(sdc, {"image": xs, "bboxes": bs}, dual_head=True)
        ref, rate, proto = cpu_baseline(sdc, xs, bs, ci["threads"], fwd=fwd)
        what = ("its own FPN level 0 -> detector glue -> heatmap head + KEYPOINT_HEAD" if detect else
                "the reference's per-box loop -> heatmap head + KEYPOINT_HEAD")
        res["cpu_baseline"] = {
            "value": round(rate, 3), "unit": "images/s", "cores": ci["threads"], "kind": "port",
            "sample": f"{S} images of the same {name} workload, oracle/kpd_oracle.py ({what}), "
                      f"{proto['warmups']} warmups + median of {proto['runs']} runs",
            "protocol": proto, "cpu_model": ci["model"]}
        res["gpu_vs_cpu"] = round(res["value"] / rate, 1)
        gk = out["keypoints"][:S].cpu()
        d = (gk - ref["keypoints"]).norm(dim=-1)
        par = {"images": S, "pck@0.5": float((d <= 0.5).float().mean()),
               "pck@0.002": float((d <= 0.002).float().mean()),
               "max_abs_dkpt": float((gk - ref["keypoints"]).abs().max()),
               "max_abs_dheat": float((out["heatmap"][:S].cpu() - ref["heatmap"]).abs().max()),
               "vis_flips": int((out["visibilities"][:S].cpu() != ref["visibilities"]).any(-1).sum()),
               "max_abs_dkh_kpt": float((out["kh_keypoints"][:S].cpu() - ref["kh_keypoints"]).abs().max()),
               "max_abs_dkh_vis": float((out["kh_visibilities"][:S].cpu() - ref["kh_visibilities"]).abs().max()),
               "kh_vis_argmax_flips": int((out["kh_visibilities"][:S].cpu().argmax(-1)
                                           != ref["kh_visibilities"].argmax(-1)).sum())}
        if detect:
            gb = torch.stack([out["boxes"][i].cpu() for i in range(S)])
            par.update({"kept_persons_equal": bool(torch.equal((out["box_scores"][:S].cpu() > 0).sum(1),
                                                               (ref["box_scores"] > 0).sum(1))),
                        "max_abs_dbox": float((gb - torch.stack(list(ref["boxes"]))).abs().max()),
                        "max_abs_dscore": float((out["box_scores"][:S].cpu() - ref["box_scores"]).abs().max())})
        res["parity"] = par
    del m, plan, out
    torch.cuda.empty_cache()
    return res


def config_names(a, world, standin=False):
    """Labelled config objects of this run: N = 1: C1 + C3 + C5; N > 1: C4 + C5
    (C1 is one image's latency on one GPU; not with the CPU stand-in)."""
    if a.only:
        return [a.only]
    if a.configs == "none":
        return []
    if a.configs == "auto":
        names = ["C1", "C3", "C5"] if world == 1 else ["C4", "C5"]
    else:
        names = [x for x in a.configs.split(",") if x]
    return [n for n in names if not (standin and n == "C1")]


def run_c1(a, dev, cpu=True):
    """BASELINE C1: scripts/predict.py's forward -- one 256x192 image, one box --
    as synchronous latency: median (and p90) of 50 forwards after 10 warm-ups,
    the same forwards replayed as hipGraphs (kpd_plan_set_graphs; outputs
    checked identical), beside the CPU reference path (the golden-pinned
    oracle, 3 warm-ups + median of 5) on this host's CPU share."""
    from dll.configs import ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    from dll.models.synthetic import synthetic_boxes, synthetic_images, synthetic_state_dict
    m = MultiPersonKeypointModel(ModelConfig(), TrainingConfig(), precision=a.precision, streams=1)
    sd = synthetic_state_dict(m.state_dict(), seed=0)
    m.load_state_dict(sd)
    m = m.to(dev).eval()
    img, box = synthetic_images(1, 3, 256, 192, seed=7), synthetic_boxes(1, 1, seed=8)
    batch = {"image": img.to(dev), "bboxes": box.to(dev)}

    def lat(n=60, skip=10):
        ts = []
        with torch.no_grad():
            for i in range(n):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                o = m(batch)
                torch.cuda.synchronize()
                if i >= skip:
                    ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts, o
    ts, out = lat()
    plan = m.native_plan(dev)
    plan.set_graphs(True)
    tg, outg = lat()
    plan.set_graphs(False)
    res = {"workload": "C1: one 256x192x3 image, one box (scripts/predict.py's forward), synchronous latency",
           "gpu_latency_ms": round(ts[len(ts) // 2] * 1e3, 4), "gpu_latency_p90_ms": round(ts[int(len(ts) * .9)] * 1e3, 4),
           "gpu_latency_graph_ms": round(tg[len(tg) // 2] * 1e3, 4),
           "graph_outputs_identical": all(torch.equal(out[k], outg[k]) for k in ("keypoints", "visibilities", "heatmap")),
           "forwards": len(ts), "warmup": 10, "precision": a.precision,
           "value": round(1.0 / ts[len(ts) // 2], 2), "unit": "images/s (1 / median latency)"}
    if cpu:
        from oracle import kpd_oracle as O
        ci = host_cpu_info()
        ref, rate, proto = cpu_baseline(sd, img, box, ci["threads"])
        res["cpu_baseline"] = {"value": round(1e3 / rate, 3), "unit": "ms/image (latency)", "cores": ci["threads"],
                               "kind": "port", "sample": f"the same image and box, oracle/kpd_oracle.py forward, "
                                                         f"{proto['warmups']} warmups + median of {proto['runs']} runs",
                               "protocol": proto, "cpu_model": ci["model"]}
        res["gpu_vs_cpu_latency"] = round(res["cpu_baseline"]["value"] / res["gpu_latency_ms"], 1)
        res["parity"] = {"max_abs_dkpt": float((out["keypoints"].cpu() - ref["keypoints"]).abs().max()),
                         "max_abs_dheat": float((out["heatmap"].cpu() - ref["heatmap"]).abs().max()),
                         "vis_flips": int((out["visibilities"].cpu() != ref["visibilities"]).any(-1).sum())}
    del m, plan, out, outg
    torch.cuda.empty_cache()
    return res


def kernel_src_hash():
    """sha256 (16 hex) over the HIP sources + headers libkpd.so is built from;
    profiles/*/pmc.json entries carry the hash they were measured on."""
    import hashlib
    h = hashlib.sha256()
    cs = ROOT / "keypoint-detection_amd" / "csrc"
    for f in sorted(list(cs.glob("*.hip")) + list(cs.glob("*.h")) + [ROOT / "include" / "kpd.h"]):
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:16]


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1 or (a.force_dist and "MASTER_ADDR" in os.environ)
    if a.cpu_standin:
        if dist:
            import torch.distributed as tdist
            tdist.init_process_group("gloo")
        return main_standin(a, world, rank, dist)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        import torch.distributed as tdist
        tdist.init_process_group("nccl", device_id=dev)

    from dll.configs import ModelConfig, TrainingConfig
    from dll.models import MultiPersonKeypointModel
    from dll.models.synthetic import synthetic_boxes, synthetic_images, synthetic_state_dict

    pmc = None
    pj = Path(a.pmc_json)
    if pj.exists():
        try:
            pmc = json.loads(pj.read_text())
        except ValueError:
            pmc = None
    if a.only:
        res = (run_c1(a, dev, cpu=not a.no_cpu_baseline) if a.only == "C1" else
               run_pipeline(a.only, a, dev, pmc, world, rank, dist, cpu=not a.no_cpu_baseline))
        if rank == 0:
            print(json.dumps({"configs": {a.only: res}}), flush=True)
        if dist:
            tdist.destroy_process_group()
        return

    def build(precision):
        m = MultiPersonKeypointModel(ModelConfig(), TrainingConfig(), precision=precision, streams=a.streams)
        m.load_state_dict(sd)
        return m.to(dev).eval()

    sd = synthetic_state_dict(MultiPersonKeypointModel(ModelConfig(), TrainingConfig()).state_dict(), seed=0)
    m = build(a.precision)
    B, P = a.batch, a.persons
    img_cpu = synthetic_images(B, 3, a.height, a.width, seed=1234 + 7919 * rank)
    box_cpu = synthetic_boxes(B, P, seed=1235 + 7919 * rank)
    img, boxes = img_cpu.to(dev), box_cpu.to(dev)
    batch = {"image": img, "bboxes": boxes}
    plan = m.native_plan(dev)

    gather = dist and not a.no_gather
    coll = {}
    pend = Collator(B * world, ("keypoints", "visibilities"), P, coll)

    def step(model=m):
        out = model(batch)
        if gather:   # result collation over RCCL: all_gather of the kpt / vis slabs (P known: no host sync)
            pend.start(out)
        return out

    n_sub = max(1, min(a.streams, 4, B // 16))
    Bl = B // n_sub if B % n_sub == 0 else B / n_sub      # images per kernel launch (one sub-batch)
    # warm-up, then one forward with every stage's events (the breakdown), then
    # the timed region with events around the dominant MFMA kernel only (no
    # bubbles elsewhere): its mean launch time is the roofline's denominator
    with torch.no_grad():
        for _ in range(a.warmup):
            step()
        pend.finish()
    breakdown = stage_pass(m, plan, batch, 1)
    mfma_stages = ("fpn0", "hm_conv1", "hm_conv2", "hm_conv3")
    dom = max((k for k in breakdown if k in mfma_stages), key=lambda k: breakdown[k][0], default=None)
    plan.timing(True, stage=dom)
    el, out = run_steps(a.steps, 0, step, dist, finish=pend.finish)
    plan.timing(False)
    dms, dn = plan.timing_query(dom) if dom else (0.0, 0)
    stages = {k: v[0] for k, v in breakdown.items()}
    if dn:
        stages[dom] = dms / dn
    per_rank = gather_elapsed(el, world, dist, dev)
    el = max(per_rank)

    fl = flops_per_image(a.height, a.width, P)
    roof = roofline(a.precision, stages, fl, Bl, a.height, a.width, pmc, dom)
    if roof:
        roof["forwards_before_timed"] = a.warmup + 1     # --warmup + the one stage-breakdown forward
        roof["launches_timed"] = dn
        roof["images_per_launch"] = Bl
        roof["timing"] = ("HIP events around every launch of this kernel inside the timed region, on the "
                          "sub-batch stream it is launched on")
    total_imgs = B * world * a.steps
    dtypes = {"split": ("fp32", "fp32-accurate: body/laterals/heads fp32; FPN level 0 and the heatmap-head convs "
                                "as 3 f16 MFMA products of hi/lo operand splits (fp32 tolerances), fp32 accumulate"),
              "fp32": ("fp32", "every conv on fp32-input MFMA (exact fp32 products)"),
              "mixed": ("bf16", "heatmap-head convs bf16 x bf16 (fp32 accumulate); backbone/FPN fp32-accurate")}
    line = {
        "metric": "images/sec @ 256x192 COCO-17 (MultiPersonKeypointModel.forward, given boxes)",
        "value": round(total_imgs / el, 2), "unit": "images/s", "n_gpus": world, "world": world,
        "backend": "nccl (RCCL)" if dist else None, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "rank_ms_per_step": [round(t / a.steps * 1e3, 4) for t in per_rank],
        "rccl_ranks": rank_census(dist, dev),
        "dtype": dtypes[a.precision][0], "dtype_detail": dtypes[a.precision][1],
        "data": "synthetic (seeded U[0,1) images ImageNet-normalised, seeded boxes, seed-0 random weights)",
        "config": {"workload": f"C2: batch {B}/GPU, {a.height}x{a.width}x3, {P} box/img, heatmap head + "
                               "soft-argmax decode",
                   "model": "MultiPersonKeypointModel (MobileNetV3-Small+FPN, HeatmapHead)",
                   "global_batch": B * world, "height": a.height, "width": a.width, "persons": P,
                   "precision": a.precision, "parallelism": f"dp{world}", "streams_per_gpu": n_sub,
                   "gather": bool(gather), "gather_pipelined": bool(gather)},
        "gflop_per_image": round(fl["total"] / 1e9, 3),
        "achieved_tflops_total": round(fl["total"] * total_imgs / el / 1e12, 2),
        "roofline": roof,
        "stages_ms": {k: round(v, 4) for k, v in stages.items()},
        "stages_note": f"per launch (one sub-batch of {Bl} images): one forward with every stage's HIP events "
                       "before the timed region; the dominant stage's figure is its timed-region mean.  Not a "
                       "partition of ms_per_step: the event-instrumented forward leaves a gap at every stage "
                       "boundary (so the stages sum to more than a step), and ms_per_step is a wall-clock mean",
        "cpu_baseline": None,
    }
    if gather:   # every rank's keypoint / visibility slab at its shard's offset in every rank's collated copy
        line["collated"] = {k: list(v.shape) for k, v in coll.items()}
        line["collated_ok"] = collation_check(out, coll, ("keypoints", "visibilities"), P, world, rank, dist, dev)
    if world == 1 and a.alt_streams and a.alt_streams != a.streams and B // 16 >= 2:
        # the same model, batch and precision as concurrent sub-batches (kpd_plan_set_streams): the
        # sub-batches' kernels overlap, so this is a throughput figure only (no per-kernel timing)
        m.streams = a.alt_streams
        el3, _ = run_steps(a.steps, a.warmup, step, False)
        m.streams = a.streams
        line["alt_streams"] = {"streams_per_gpu": max(1, min(a.alt_streams, 4, B // 16)),
                               "value": round(B * a.steps / el3, 2), "ms_per_step": round(el3 / a.steps * 1e3, 4),
                               "precision": a.precision}
    if world == 1 and a.secondary and a.secondary != a.precision:
        # the same workload at the second precision (labelled; not the headline)
        m2 = build(a.secondary)
        p2 = m2.native_plan(dev)
        with torch.no_grad():
            for _ in range(a.warmup):
                step(m2)
        bd2 = stage_pass(m2, p2, batch, 1)
        d2 = max((k for k in bd2 if k in mfma_stages), key=lambda k: bd2[k][0], default=None)
        p2.timing(True, stage=d2)
        el2, _ = run_steps(a.steps, 0, lambda: step(m2), False)
        p2.timing(False)
        st2 = {k: v[0] for k, v in bd2.items()}
        if d2:
            ms2, n2 = p2.timing_query(d2)
            if n2:
                st2[d2] = ms2 / n2
        line["secondary"] = {"precision": a.secondary, "dtype": dtypes[a.secondary][0],
                             "dtype_detail": dtypes[a.secondary][1], "value": round(B * a.steps / el2, 2),
                             "ms_per_step": round(el2 / a.steps * 1e3, 4),
                             "roofline": roofline(a.secondary, st2, fl, Bl, a.height, a.width, pmc, d2),
                             "stages_ms": {k: round(v, 4) for k, v in st2.items()}}
        del m2, p2
    if world == 1 and a.exact_check and a.precision != "fp32":
        # cross-check of the headline precision: the same batch through the exact-product fp32 mode
        # (every conv on fp32-input MFMA), its throughput and its distance from the headline outputs
        m3 = build("fp32")
        with torch.no_grad():
            for _ in range(3):
                out3 = step(m3)
        n3 = max(1, min(a.steps, 10))
        el4, out3 = run_steps(n3, 0, lambda: step(m3), False)
        line["exact_fp32"] = {
            "precision": "fp32", "dtype_detail": dtypes["fp32"][1], "steps": n3,
            "value": round(B * n3 / el4, 2), "ms_per_step": round(el4 / n3 * 1e3, 4),
            "vs_headline": {
                "max_abs_dkpt": float((out3["keypoints"] - out["keypoints"]).abs().max()),
                "max_abs_dheat": float((out3["heatmap"] - out["heatmap"]).abs().max()),
                "vis_flips": int((out3["visibilities"].argmax(-1) != out["visibilities"].argmax(-1)).sum()),
                "keypoints_compared": int(out["keypoints"][..., 0].numel())},
            "note": "same batch and weights as the headline; the headline's split products against exact fp32 "
                    "products (tolerances of the parity tests: 1e-5 keypoints, 5e-5 heatmaps)"}
        del m3
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        ci = host_cpu_info()
        S = min(a.cpu_sample, B)
        ref, cpu_rate, proto = cpu_baseline(sd, img_cpu[:S], box_cpu[:S], ci["threads"])
        line["cpu_baseline"] = {
            "value": round(cpu_rate, 3), "unit": "images/s", "cores": ci["threads"], "kind": "port",
            "sample": f"{S} images of the same C2 workload, oracle/kpd_oracle.py forward (the reference's per-box "
                      f"loop, golden-pinned), {proto['warmups']} warmups + median of {proto['runs']} runs",
            "protocol": proto, "cpu_model": ci["model"], "machine_physical_cores": ci["physical_cores"],
            "machine_logical_cpus": ci["logical_cpus"], "cgroup_cpu_quota": ci["cgroup_cpus"],
            "threads_note": "torch threads = min(affinity, cgroup cpu.max quota, physical cores): the CPU share "
                            "this job may use on the GPU box"}
        line["gpu_vs_cpu"] = round(line["value"] / cpu_rate, 1)
        gk = out["keypoints"][:S].cpu()
        d = (gk - ref["keypoints"]).norm(dim=-1)
        line["parity"] = {"pck@0.5": float((d <= 0.5).float().mean()), "pck@0.002": float((d <= 0.002).float().mean()),
                          "max_abs_dkpt": float((gk - ref["keypoints"]).abs().max()),
                          "max_abs_dheat": float((out["heatmap"][:S].cpu() - ref["heatmap"]).abs().max()),
                          "vis_flips": int((out["visibilities"][:S].cpu() != ref["visibilities"]).any(-1).sum()),
                          "images": S}
    names = config_names(a, world)
    if names:
        # the north_star's full pipeline (C3 at N=1, C4 at N>1) and C5 as labelled objects beside the C2
        # headline, on the same ranks
        del m, plan
        torch.cuda.empty_cache()
        line["configs"] = {n: (run_c1(a, dev, cpu=not a.no_cpu_baseline) if n == "C1" else
                               run_pipeline(n, a, dev, pmc, world, rank, dist, cpu=not a.no_cpu_baseline))
                           for n in names}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
