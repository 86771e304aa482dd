"""Generate golden vectors by running the REFERENCE's own Python code.

Runs only in the build container (needs /root/reference).  Imports the
reference modules from /root/reference/dll without executing its package
__init__ (which would import cv2/the data pipeline): ``dll`` and ``dll.models``
are registered as namespace packages pointing at the reference directories,
bytecode writing is disabled, and the absent torchvision pieces come from
tests/golden/tv_shim.py (restated, see there).

Fixtures (tests/golden/*.npz) hold inputs' seeds/checksums and the reference
outputs; weights are regenerated from seed 0 by
dll.models.synthetic.synthetic_state_dict and pinned by a checksum.

    python -B tests/golden/make_golden.py
"""
from __future__ import annotations

import sys
import types
from pathlib import Path

sys.dont_write_bytecode = True
ROOT = Path(__file__).resolve().parents[2]
REF = Path("/root/reference")
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "golden"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import tv_shim  # noqa: E402

OUT = ROOT / "tests" / "golden"


def import_reference():
    tv_shim.install()
    # product package lives under keypoint-detection_amd/dll -- keep it out of
    # the way: the reference's 'dll' namespace is registered explicitly.
    pkg = types.ModuleType("dll")
    pkg.__path__ = [str(REF / "dll")]
    sys.modules["dll"] = pkg
    models = types.ModuleType("dll.models")
    models.__path__ = [str(REF / "dll" / "models")]
    sys.modules["dll.models"] = models
    import dll.configs as rc  # noqa: F401
    from dll.models.keypoint_model import MultiPersonKeypointModel
    from dll.models.person_head import PERSON_HEAD
    from dll.models.heatmap_head import HeatmapHead, decode_heatmaps, decode_heatmaps_soft_argmax
    from dll.models.keypoint_head import KEYPOINT_HEAD
    return types.SimpleNamespace(cfg=rc, Model=MultiPersonKeypointModel, PersonHead=PERSON_HEAD,
                                 HeatmapHead=HeatmapHead, KeypointHead=KEYPOINT_HEAD,
                                 decode_heatmaps=decode_heatmaps, decode_sa=decode_heatmaps_soft_argmax)


def load_synthetic():
    """Import the product's synthetic helpers by file path (the name 'dll' is
    taken by the reference namespace here)."""
    import importlib.util
    p = ROOT / "keypoint-detection_amd" / "dll" / "models" / "synthetic.py"
    spec = importlib.util.spec_from_file_location("kpd_synthetic", p)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def build_model(R, S, in_channels=3):
    cfg = R.cfg.ModelConfig(backbone=R.cfg.BackboneConfig(in_channels=in_channels))
    m = R.Model(cfg, R.cfg.TrainingConfig())
    sd = S.synthetic_state_dict(m.state_dict(), seed=0)
    m.load_state_dict(sd, strict=True)
    m.eval()
    return m, sd


def run_case(m, image, bboxes):
    with torch.no_grad():
        feats = m.backbone(image)[0]
        scores = m.channel_attention(feats)
        out = m({"image": image, "bboxes": bboxes})
    return feats, scores, out


def main():
    R = import_reference()
    S = load_synthetic()
    torch.manual_seed(0)
    m3, sd3 = build_model(R, S, 3)
    np.savez_compressed(OUT / "weights_fingerprint.npz",
                        keys=np.array(sorted(sd3.keys())),
                        checksum=np.array(S.weights_checksum(sd3)))

    # ---- case main: B=2, 3x256x192, P=3 with an all-zero box in image 1
    img = S.synthetic_images(2, 3, 256, 192, seed=1234)
    boxes = S.synthetic_boxes(2, 3, seed=1235)
    boxes[1, 1] = 0.0
    feats, scores, out = run_case(m3, img, boxes)
    topk = torch.topk(scores, 64, dim=1).indices
    hm = out["heatmap"]
    np.savez_compressed(
        OUT / "forward_main.npz",
        image_sum=img.double().sum().numpy(), boxes=boxes.numpy(),
        feat0_chan_mean=feats.mean(dim=(2, 3)).numpy(), feat0_chan_max=feats.amax(dim=(2, 3)).numpy(),
        feat0_slice=feats[:, :, 60:64, 40:44].numpy(),
        scores=scores.numpy(), topk=topk.numpy(),
        keypoints=out["keypoints"].numpy(), visibilities=out["visibilities"].numpy(),
        heatmap_sum=hm.double().sum(dim=(3, 4)).numpy(), heatmap_max=hm.amax(dim=(3, 4)).numpy(),
        heatmap_b0p0=hm[0, 0].numpy())
    print("main", out["keypoints"].shape, out["visibilities"].shape, hm.shape)

    # ---- case dummy: one image whose only boxes are all zero; P=2
    b2 = torch.zeros(2, 2, 4)
    b2[0] = S.synthetic_boxes(1, 2, seed=7)[0]
    _, _, out = run_case(m3, img, b2)
    np.savez_compressed(OUT / "forward_dummy.npz", boxes=b2.numpy(), keypoints=out["keypoints"].numpy(),
                        visibilities=out["visibilities"].numpy(),
                        heatmap_sum=out["heatmap"].double().sum(dim=(3, 4)).numpy())
    print("dummy", out["visibilities"][1, :, 0, :2])

    # ---- case empty: P = 0 -> zeros, 2-D visibilities
    _, _, out = run_case(m3, img, torch.zeros(2, 0, 4))
    np.savez_compressed(OUT / "forward_empty.npz", kshape=np.array(out["keypoints"].shape),
                        vshape=np.array(out["visibilities"].shape), hshape=np.array(out["heatmap"].shape))
    print("empty", out["keypoints"].shape, out["visibilities"].shape)

    # ---- case list input [P,4] -> single image (list branch, :97-103); grayscale 224x224 like predict.py
    m1, _ = build_model(R, S, 1)
    img1 = S.synthetic_images(1, 1, 224, 224, seed=99)
    bl = S.synthetic_boxes(1, 2, seed=100)[0]
    _, sc1, out = run_case(m1, img1, [bl])
    np.savez_compressed(OUT / "forward_gray_list.npz", boxes=bl.numpy(), scores=sc1.numpy(),
                        keypoints=out["keypoints"].numpy(), visibilities=out["visibilities"].numpy(),
                        heatmap_sum=out["heatmap"].double().sum(dim=(3, 4)).numpy())
    print("gray", out["keypoints"].shape)

    # ---- NMS known answers (person_head.py:96-139)
    ph = R.PersonHead(R.cfg.PersonDetectionConfig())
    g = torch.Generator().manual_seed(5)
    cases = []
    for n, thr, mo in [(40, 0.3, None), (40, 0.5, 5), (200, 0.3, None), (200, 0.2, 10), (1, 0.3, None)]:
        bx = torch.rand(n, 4, generator=g)
        bx[:, 2:] = bx[:, 2:] * 0.3 + 0.05
        sc = torch.rand(n, generator=g)
        if n >= 40:
            sc[5] = sc[7]  # an exact tie
        keep = ph.non_max_suppression(bx, sc, thr, mo)
        cases.append((bx.numpy(), sc.numpy(), thr, -1 if mo is None else mo, keep.numpy()))
    np.savez_compressed(OUT / "nms.npz", **{f"c{i}_{k}": v for i, c in enumerate(cases)
                                             for k, v in zip(("boxes", "scores", "thr", "max_out", "keep"), c)})
    iou = ph.box_iou(torch.tensor(cases[0][0][:6]), torch.tensor(cases[0][0][:9]))
    np.savez_compressed(OUT / "box_iou.npz", b1=cases[0][0][:6], b2=cases[0][0][:9], iou=iou.numpy())
    print("nms keeps", [len(c[4]) for c in cases])

    # ---- HeatmapHead standalone + decode helpers
    hh = R.HeatmapHead(R.cfg.HeatmapHeadConfig())
    hsd = {k[len("heatmap_head."):]: v for k, v in sd3.items() if k.startswith("heatmap_head.")}
    hh.load_state_dict(hsd)
    hh.eval()
    xr = torch.randn(1, 64, 56, 56, generator=g).half().float()
    with torch.no_grad():
        hmap, _ = hh(xr)
        dk, ds = R.decode_heatmaps(hmap)
        sk, ss = R.decode_sa(hmap)
        kk, kv = m3.decode_heatmap(hmap)
        ka = m3._soft_argmax(hmap)
    np.savez_compressed(OUT / "heatmap_head.npz", x_seed=np.array(5), x=xr.numpy().astype(np.float16),
                        heat_sum=hmap.double().sum(dim=(2, 3)).numpy(), heat_slice=hmap[:, :, 20:24, 30:34].numpy(),
                        argmax_kpts=dk.numpy(), argmax_scores=ds.numpy(), sa_kpts=sk.numpy(), sa_scores=ss.numpy(),
                        model_kpts=kk.numpy(), model_vis=kv.numpy(), model_softargmax=ka.numpy())

    # ---- KEYPOINT_HEAD standalone (the 'dual head'); config from the YAML (56x56)
    kcfg = R.cfg.KeypointHeadConfig(height=56, width=56)
    kh = R.KeypointHead(kcfg)
    ksd = S.synthetic_state_dict(kh.state_dict(), seed=3)
    kh.load_state_dict(ksd)
    kh.eval()
    xk = torch.randn(2, 128, 56, 56, generator=torch.Generator().manual_seed(11))
    with torch.no_grad():
        kp, kvv = kh(xk)
    np.savez_compressed(OUT / "keypoint_head.npz", keypoints=kp.numpy(), visibility=kvv.numpy(),
                        checksum=np.array(S.weights_checksum(ksd)))
    print("done")


if __name__ == "__main__":
    main()
