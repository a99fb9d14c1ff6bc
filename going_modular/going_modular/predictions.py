"""Reference-compatible ``predictions`` (GM/predictions.py): pred_and_plot_image."""
from pytorch_vit_paper_replication_amd.predictions import device, pred_and_plot_image, predict_image  # noqa: F401
