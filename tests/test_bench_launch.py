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
    r = _run(["--gpus", "2", "--cpu-standin", "--steps", "3", "--warmup", "1", "--batch", "6", "--persons", "2"])
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 2 and line["world"] == 2 and line["backend"] == "gloo"
    assert len(line["rank_ms_per_step"]) == 2
    assert line["ms_per_step"] == max(line["rank_ms_per_step"])
    assert line["collated"]["keypoints"] == [12, 2, 1, 17, 2]
    assert line["collated"]["visibilities"] == [12, 2, 1, 17, 3]
    assert line["collated_ok"] is True


def test_bench_gpus1_single_process():
    r = _run(["--gpus", "1", "--cpu-standin", "--steps", "2", "--warmup", "0", "--batch", "4"])
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 1 and line["world"] == 1 and line["collated"] == {}


def test_bench_gpus_mismatch_fails():
    """Under a launcher, --gpus must equal WORLD_SIZE."""
    r = _run(["--gpus", "4", "--cpu-standin", "--steps", "1"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr
