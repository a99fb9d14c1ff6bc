"""The course's ``helper_functions`` used by the reference notebooks (MAIN.ipynb:81, :90).

``download_data`` cannot reach the network here: it returns an existing local directory or raises
with instructions (synthetic data: ``pytorch_vit_paper_replication_amd.data``)."""
from pathlib import Path

from pytorch_vit_paper_replication_amd.utils.plotting import plot_loss_curves  # noqa: F401
from pytorch_vit_paper_replication_amd.utils.seed import set_seeds  # noqa: F401


def download_data(source: str, destination: str, remove_source: bool = True) -> Path:
    data_path = Path("data/")
    image_path = data_path / destination
    if image_path.is_dir():
        print(f"[INFO] {image_path} directory exists, skipping download.")
        return image_path
    raise RuntimeError(f"No network access: place the dataset at {image_path} (expected <split>/<class>/<img>) "
                       f"or use synthetic data (pytorch_vit_paper_replication_amd.data.create_synthetic_dataloaders).")
