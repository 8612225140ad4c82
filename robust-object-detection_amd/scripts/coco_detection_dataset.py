"""Drop-in for the reference's scripts/coco_detection_dataset.py (COCO json -> (image, target))."""
from mx_det.dataset import COCODetectionDataset, collate_fn  # noqa: F401
