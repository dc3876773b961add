"""MI355X-native (gfx950 / CDNA4) training path for 3D multimodal organ
segmentation — a drop-in for the training hot path of
wittyseok/multimodal-organ-segmentation (build_model / Trainer.train_step).

Import as `mmseg_amd` (the repo-root shim maps that name onto this directory).
"""
__version__ = "0.1.0"
