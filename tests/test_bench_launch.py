"""bench.py's N-rank branch on the CPU: `python bench.py --gpus 2` (no
launcher) must start 2 ranks itself through torch.distributed.run, time the
steps between barriers, take the max over ranks and collate the per-image
slabs with all_gather -- here over gloo with --cpu-standin's stand-in forward
(the same launcher, timing and collation code the RCCL run uses)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=env, capture_output=True, text=True,
                          timeout=240, cwd=str(ROOT))


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks():
    """N = 2: the C2 headline plus the C4 (C3 pipeline per rank, detector
    outputs collated) and C5 (given boxes, dual head) objects, each timed
    between barriers with the max over ranks and every rank's slab found at
    its shard's offset in the collated outputs."""
    r = _run(["--gpus", "2", "--cpu-standin", "--steps", "3", "--warmup", "1", "--batch", "6", "--persons", "2",
              "--cfg-batch", "3"])
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 2 and line["world"] == 2 and line["backend"] == "gloo"
    assert len(line["rank_ms_per_step"]) == 2
    assert line["ms_per_step"] == max(line["rank_ms_per_step"])
    assert line["collated"]["keypoints"] == [12, 2, 1, 17, 2]
    assert line["collated"]["visibilities"] == [12, 2, 1, 17, 3]
    assert line["collated_ok"] is True and line["collated_index_ok"] is True
    assert line["rccl_ranks"] == 2
    cfg = line["configs"]
    assert sorted(cfg) == ["C4", "C5"]
    c4, c5 = cfg["C4"], cfg["C5"]
    for c in (c4, c5):
        assert c["n_gpus"] == 2 and c["global_batch"] == 6 and c["images_per_rank"] == 3
        assert len(c["rank_ms_per_step"]) == 2 and c["ms_per_step"] == max(c["rank_ms_per_step"])
        assert c["collated_ok"] is True and c["collated_index_ok"] is True and c["rccl_ranks"] == 2
        assert c["collated"]["keypoints"] == [6, 5, 1, 17, 2]
        assert c["collated"]["kh_visibilities"] == [6, 5, 1, 17, 3]
    assert c4["collated"]["boxes"] == [6, 5, 4] and c4["collated"]["box_scores"] == [6, 5]
    assert "boxes" not in c5["collated"] and "384x288" in c5["workload"]


def test_bench_gpus1_single_process():
    r = _run(["--gpus", "1", "--cpu-standin", "--steps", "2", "--warmup", "0", "--batch", "4", "--cfg-batch", "2"])
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 1 and line["world"] == 1 and line["collated"] == {} and line["rccl_ranks"] is None
    assert sorted(line["configs"]) == ["C3", "C5"]
    assert all("collated" not in c for c in line["configs"].values())


def test_bench_gpus_mismatch_fails():
    """Under a launcher, --gpus must equal WORLD_SIZE."""
    r = _run(["--gpus", "4", "--cpu-standin", "--steps", "1"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr
