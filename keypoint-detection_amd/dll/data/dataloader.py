"""YOLO-pose dataset, collate and loaders -- drop-in for the reference's
``dll/data/dataloader.py`` feeding the MI355X path.

What runs where:

* host: directory scan, image decode (Pillow), label text parsing (numpy);
* device: ``ITransform`` (``kpd_preprocess``) and the target heatmaps
  (``kpd_target_heatmaps``), so a sample's ``image`` and ``heatmaps`` are
  already resident on the GPU;
* collate: padding copies into device tensors (plumbing).

Semantics follow the reference line by line, quirks included (pinned by
tests/golden/data.npz, produced by the reference's own methods):

* label rows are padded with zeros to the longest row, keypoint columns padded
  or truncated to 3*num_keypoints, visibility truncated to int
  (``_parse_label_file_vectorized`` :199-257); any parse error yields the
  empty annotation;
* persons need a visible keypoint and a non-zero coordinate (:275-306); the box
  tensor is masked only when it holds more than one box;
* ``AnnotationData`` keeps keypoints as [1, P, K, 2], so ``num_persons`` is 1
  and ``truncate`` does not cut persons (:36-49); the target heatmap is the
  first person's (generate_target_heatmap flattens B*P but loops over B); and
  the collate keeps the first person of every image (:432-560).

Differences: images are decoded by Pillow, not ``cv2.imread`` (the JPEG
decoders may differ by a grey level; cv2 is absent here), and DataLoader
workers are not used when the dataset runs on a GPU (forked workers cannot
share the HIP context) -- the GPU stages are fast enough not to need them.
Training augmentation (``KeypointAugmentation``) is out of scope.
"""
from __future__ import annotations

import logging
from collections import OrderedDict
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

from ..models.heatmap_head import generate_target_heatmap
from .transforms import ITransform

logger = logging.getLogger(__name__)

IMG_EXTENSIONS = (".png", ".jpg", ".jpeg")


class KeypointDatasetError(Exception):
    """Dataset errors (same class names as the reference, :22-28)."""


class ValidationError(KeypointDatasetError):
    pass


@dataclass
class AnnotationData:
    keypoints: torch.Tensor       # [1, P, K, 2]
    visibilities: torch.Tensor    # [1, P, K]
    classes: torch.Tensor         # [P]
    bboxes: Any                   # list holding one [P, 4] tensor

    def truncate(self, max_persons: int) -> "AnnotationData":
        # slices the leading axis, which is the singleton one (reference :39-45)
        return AnnotationData(self.keypoints[:max_persons], self.visibilities[:max_persons],
                              self.classes[:max_persons], self.bboxes[:max_persons])

    @property
    def num_persons(self) -> int:
        return self.keypoints.shape[0]


@dataclass
class ImageData:
    image: Any                    # PIL image
    orig_size: Tuple[int, int]    # (width, height)


class LRUCache:
    def __init__(self, maxsize: int = 128):
        self.cache: "OrderedDict[Any, Any]" = OrderedDict()
        self.maxsize = maxsize

    def get(self, key: Any) -> Any:
        v = self.cache.get(key)
        if v is not None:
            self.cache.move_to_end(key)
        return v

    def put(self, key: Any, value: Any) -> None:
        if key in self.cache:
            self.cache.move_to_end(key)
        elif len(self.cache) >= self.maxsize:
            self.cache.popitem(last=False)
        self.cache[key] = value


class OptimizedKeypointsDataset(Dataset):
    """``<dataset_dir>/<split>/{images,labels}`` with YOLO-pose label files
    (``cls cx cy w h  x1 y1 v1 ... xK yK vK``, normalised)."""

    def __init__(self, dataset_dir: str, split: str = "train", img_size: int = 512, grayscale: bool = False,
                 num_keypoints: int = 17, heatmap_size: Tuple[int, int] = (56, 56),
                 transform: Optional[ITransform] = None, augmentation=None, max_persons: int = 10,
                 enable_caching: bool = True, cache_size: int = 1000,
                 device: Union[str, torch.device] = "cuda"):
        self.dataset_dir = Path(dataset_dir)
        self.split = split
        self.img_size = img_size
        self.grayscale = grayscale
        self.num_keypoints = num_keypoints
        self.heatmap_size = heatmap_size
        self.max_persons = max_persons
        self.enable_caching = enable_caching
        self.device = torch.device(device)
        self._annotation_cache = {} if enable_caching else None
        self._image_cache = LRUCache(maxsize=cache_size) if enable_caching else None
        self.transform = transform or ITransform(img_size=img_size, clip_limit=1.5, tile_size=(8, 8),
                                                 grayscale=grayscale, device=self.device)
        self.augmentation = augmentation if split == "train" else None
        if self.augmentation is not None:
            raise NotImplementedError("training augmentation is out of scope for the MI355X data path")
        self._validate_dataset_structure()
        self.img_files, self.label_files = self._load_file_pairs()
        logger.info(f"Loaded {len(self.img_files)} images with valid labels for {split} split")

    # ---- files
    def _validate_dataset_structure(self) -> None:
        self.img_dir = self.dataset_dir / self.split / "images"
        self.label_dir = self.dataset_dir / self.split / "labels"
        for d, what in ((self.img_dir, "Image"), (self.label_dir, "Label")):
            if not d.exists():
                raise KeypointDatasetError(f"{what} directory not found: {d}")

    def _load_file_pairs(self) -> Tuple[Tuple[Path, ...], Tuple[Path, ...]]:
        imgs, labels = [], []
        for img in sorted(f for f in self.img_dir.glob("*") if f.suffix.lower() in IMG_EXTENSIONS):
            lab = self.label_dir / f"{img.stem}.txt"
            if lab.exists():
                imgs.append(img)
                labels.append(lab)
            else:
                logger.warning(f"No label file found for {img}")
        if not imgs:
            raise KeypointDatasetError(f"No valid image-label pairs found in {self.dataset_dir}")
        return tuple(imgs), tuple(labels)

    def _get_file_paths(self, idx: int) -> Tuple[Path, Path]:
        if idx >= len(self.img_files):
            raise KeypointDatasetError(f"Index {idx} out of range")
        return self.img_files[idx], self.label_files[idx]

    def _load_and_process_image(self, img_path: Path) -> ImageData:
        if self._image_cache:
            hit = self._image_cache.get(str(img_path))
            if hit is not None:
                return hit
        from PIL import Image
        try:
            with Image.open(img_path) as im:
                img = im.convert("L" if self.grayscale else "RGB")
        except OSError as e:
            raise KeypointDatasetError(f"Failed to load image {img_path}") from e
        data = ImageData(image=img, orig_size=img.size)
        if self._image_cache:
            self._image_cache.put(str(img_path), data)
        return data

    # ---- labels
    def _create_empty_annotation(self) -> AnnotationData:
        K = self.num_keypoints
        return AnnotationData(keypoints=torch.zeros(1, 1, K, 2), visibilities=torch.zeros(1, 1, K),
                              classes=torch.zeros(1, dtype=torch.long), bboxes=[torch.zeros(1, 4)])

    def _parse_label_file_vectorized(self, label_path: Path) -> AnnotationData:
        try:
            with open(label_path) as f:
                rows = [[float(tok) for tok in line.split()] for line in f]
            if not rows:
                return self._create_empty_annotation()
            width = max(len(r) for r in rows)
            m = np.zeros((len(rows), width), np.float32)
            for i, r in enumerate(rows):
                m[i, :len(r)] = r
            classes = m[:, 0].astype(np.int32)          # IndexError on all-blank files, as in the reference
            boxes = m[:, 1:5]
            need = self.num_keypoints * 3
            kcols = m[:, 5:].astype(np.float64)
            if kcols.shape[1] < need:
                kcols = np.concatenate([kcols, np.zeros((len(rows), need - kcols.shape[1]))], axis=1)
            trip = kcols[:, :need].reshape(len(rows), self.num_keypoints, 3)
            return AnnotationData(
                keypoints=torch.from_numpy(trip[:, :, :2]).float().unsqueeze(0),
                visibilities=torch.from_numpy(trip[:, :, 2].astype(np.int32)).float().unsqueeze(0),
                classes=torch.from_numpy(classes).long(),
                bboxes=[torch.from_numpy(boxes).float()])
        except Exception as e:   # the reference maps every parse failure to the empty annotation
            logger.error(f"Error parsing {label_path}: {e}")
            return self._create_empty_annotation()

    def _get_annotation_data(self, label_path: Path) -> AnnotationData:
        key = str(label_path)
        if self.enable_caching and key in self._annotation_cache:
            return self._annotation_cache[key]
        ann = self._parse_label_file_vectorized(label_path)
        if self.enable_caching:
            self._annotation_cache[key] = ann
        return ann

    def _filter_valid_persons(self, ann: AnnotationData) -> AnnotationData:
        kp = ann.keypoints.squeeze(0) if ann.keypoints.dim() == 4 else ann.keypoints
        vis = ann.visibilities.squeeze(0) if ann.keypoints.dim() == 4 else ann.visibilities
        keep = (vis.sum(dim=-1) > 0) & (kp != 0).flatten(1).any(dim=1)
        if not bool(keep.any()):
            return self._create_empty_annotation()
        boxes = [b[keep] if b.size(0) > 1 else b for b in ann.bboxes]
        return AnnotationData(kp[keep].unsqueeze(0), vis[keep].unsqueeze(0), ann.classes[keep], boxes)

    # ---- sample
    def _apply_transformations(self, image_data: ImageData, ann: AnnotationData):
        return self.transform.transform(image_data.image), ann

    def _generate_training_targets(self, ann: AnnotationData) -> torch.Tensor:
        heat = generate_target_heatmap(ann.keypoints.to(self.device), self.heatmap_size, sigma=3.0)
        return heat.unsqueeze(0) if heat.dim() == 3 else heat

    def _validate_sample_data(self, ann: AnnotationData, heatmaps: torch.Tensor, img_path: Path) -> None:
        if not isinstance(ann.bboxes, list):
            raise ValidationError(f"Invalid bboxes format: expected list, got {type(ann.bboxes)}")
        for b in ann.bboxes:
            if not isinstance(b, torch.Tensor):
                raise ValidationError(f"Invalid bbox type: expected tensor, got {type(b)}")
            if b.dim() != 2 or b.size(1) != 4:
                raise ValidationError(f"Invalid bbox shape: expected [N, 4], got {tuple(b.shape)}")
        if ann.keypoints.dim() != 4:
            raise ValidationError(f"Invalid keypoints shape: expected 4D, got {ann.keypoints.dim()}D")
        if ann.visibilities.dim() != 3:
            raise ValidationError(f"Invalid visibilities shape: expected 3D, got {ann.visibilities.dim()}D")

    def _create_sample_dict(self, image: torch.Tensor, ann: AnnotationData, heatmaps: torch.Tensor,
                            img_path: Path, orig_size: Tuple[int, int]) -> Dict:
        return {"image": image, "heatmaps": heatmaps, "visibilities": ann.visibilities,
                "bboxes": ann.bboxes[0] if isinstance(ann.bboxes, list) else ann.bboxes,
                "keypoints": ann.keypoints, "num_persons": ann.num_persons, "img_path": str(img_path),
                "orig_size": orig_size}

    def __len__(self) -> int:
        return len(self.img_files)

    def __getitem__(self, idx: int) -> Dict:
        img_path, label_path = self._get_file_paths(idx)
        image_data = self._load_and_process_image(img_path)
        ann = self._filter_valid_persons(self._get_annotation_data(label_path))
        if ann.num_persons > self.max_persons:
            ann = ann.truncate(self.max_persons)
        image, ann = self._apply_transformations(image_data, ann)
        heatmaps = self._generate_training_targets(ann)
        try:
            self._validate_sample_data(ann, heatmaps, img_path)
        except ValidationError as e:
            logger.error(f"Validation error for sample {img_path}: {e}")
            raise
        return self._create_sample_dict(image, ann, heatmaps, img_path, image_data.orig_size)


def efficient_collate_fn(batch: List[Dict]) -> Dict[str, Union[torch.Tensor, List]]:
    """Pad per-image annotations to the batch's largest ``num_persons``
    (reference :432-560, the no-DeviceManager branch: everything on the first
    image's device).  Heatmap planes are fixed at 17 x 56 x 56 there too."""
    device = batch[0]["image"].device if batch else torch.device("cpu")
    paths = lambda ss: [s["img_path"] for s in ss]       # noqa: E731
    sizes = lambda ss: [s["orig_size"] for s in ss]      # noqa: E731
    valid = [s for s in batch if s["num_persons"] > 0]
    if not valid:
        n = len(batch)
        return {"image": torch.stack([s["image"].to(device) for s in batch]),
                "heatmaps": torch.zeros(n, 1, 17, 56, 56, device=device),
                "visibilities": torch.zeros(n, 1, 17, device=device),
                "bboxes": [torch.zeros(n, 1, 4, device=device)],
                "num_persons": torch.zeros(n, device=device, dtype=torch.long),
                "img_path": paths(batch), "orig_size": sizes(batch),
                "keypoints": torch.zeros(n, 1, 17, 2, device=device)}
    B = len(valid)
    P = max(s["num_persons"] for s in valid)
    heat = torch.zeros(B, P, 17, 56, 56, device=device)
    vis = torch.zeros(B, P, 17, device=device)
    boxes = torch.zeros(B, P, 4, device=device)
    kps = torch.zeros(B, P, 17, 2, device=device)
    for b, s in enumerate(valid):
        n = s["num_persons"]
        if n <= 0:
            continue
        heat[b, :n] = s["heatmaps"].to(device)[:n]
        v = s["visibilities"].to(device)
        vis[b, :n] = (v.squeeze(0) if v.dim() == 3 else v)[:n]
        bx = s["bboxes"][0] if isinstance(s["bboxes"], list) else s["bboxes"]
        bx = bx.to(device)
        if bx.dim() == 2:
            boxes[b, :n] = bx[:n]
        elif bx.dim() == 3:
            boxes[b, :n] = bx.squeeze(0)[:n]
        if "keypoints" in s:
            k = s["keypoints"].to(device)
            kps[b, :n] = (k.squeeze(0) if k.dim() == 4 else k)[:n]
    return {"image": torch.stack([s["image"].to(device) for s in valid]), "heatmaps": heat, "visibilities": vis,
            "bboxes": [boxes], "num_persons": torch.tensor([s["num_persons"] for s in valid], device=device),
            "img_path": paths(valid), "orig_size": sizes(valid), "keypoints": kps}


def _workers(num_workers: int, device: torch.device) -> int:
    if num_workers > 0 and device.type == "cuda":
        logger.info("GPU-resident dataset: DataLoader workers disabled (num_workers=0)")
        return 0
    return num_workers


def create_optimized_dataloader(dataset_dir: str, batch_size: int = 32, num_workers: int = 4, split: str = "train",
                                img_size: int = 224, grayscale: bool = True, num_keypoints: int = 17,
                                heatmap_size: Tuple[int, int] = (56, 56), max_persons: int = 10,
                                enable_caching: bool = True, cache_size: int = 1000,
                                device: Union[str, torch.device] = "cuda") -> DataLoader:
    """Reference :562-612 (same arguments; ``device`` added)."""
    ds = OptimizedKeypointsDataset(dataset_dir=dataset_dir, split=split, img_size=img_size, grayscale=grayscale,
                                   num_keypoints=num_keypoints, heatmap_size=heatmap_size,
                                   max_persons=max_persons, enable_caching=enable_caching, cache_size=cache_size,
                                   device=device)
    nw = _workers(num_workers, ds.device)
    kw = dict(batch_size=batch_size, shuffle=(split == "train"), num_workers=nw, pin_memory=False,
              drop_last=(split == "train"), collate_fn=efficient_collate_fn, persistent_workers=nw > 0)
    if nw > 0:
        kw["prefetch_factor"] = 2
    return DataLoader(ds, **kw)


class AdaptiveBatchSampler:
    """Batches of similar person counts (reference :615-675)."""

    def __init__(self, dataset: OptimizedKeypointsDataset, batch_size: int = 32, max_persons_per_batch: int = 50):
        self.dataset = dataset
        self.batch_size = batch_size
        self.max_persons_per_batch = max_persons_per_batch
        self.indices = list(range(len(dataset)))
        self.person_counts = self._compute_person_counts()

    def _compute_person_counts(self) -> List[int]:
        counts = []
        for idx in range(len(self.dataset)):
            try:
                _, lab = self.dataset._get_file_paths(idx)
                ann = self.dataset._filter_valid_persons(self.dataset._get_annotation_data(lab))
                counts.append(min(ann.num_persons, self.dataset.max_persons))
            except Exception as e:   # noqa: BLE001 -- the reference defaults to one person
                logger.warning(f"Error counting persons for sample {idx}: {e}")
                counts.append(1)
        return counts

    def __iter__(self):
        cur, persons = [], 0
        for idx in sorted(self.indices, key=lambda i: self.person_counts[i]):
            c = self.person_counts[idx]
            if cur and (len(cur) >= self.batch_size or persons + c > self.max_persons_per_batch):
                yield cur
                cur, persons = [], 0
            cur.append(idx)
            persons += c
        if cur:
            yield cur

    def __len__(self) -> int:
        return (len(self.indices) + self.batch_size - 1) // self.batch_size


def create_adaptive_dataloader(dataset_dir: str, batch_size: int = 32, num_workers: int = 4, split: str = "train",
                               max_persons_per_batch: int = 50, **dataset_kwargs) -> DataLoader:
    """Reference :678-713."""
    ds = OptimizedKeypointsDataset(dataset_dir=dataset_dir, split=split, **dataset_kwargs)
    nw = _workers(num_workers, ds.device)
    return DataLoader(ds, batch_sampler=AdaptiveBatchSampler(ds, batch_size, max_persons_per_batch),
                      num_workers=nw, pin_memory=False, collate_fn=efficient_collate_fn,
                      persistent_workers=nw > 0)
