"""``set_seeds`` of the course's helper_functions (used throughout MAIN.ipynb, e.g. :1434, :2605)."""
import random

import numpy as np
import torch


def set_seeds(seed: int = 42):
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)


def set_all_seeds(seed: int = 42):
    set_seeds(seed)
    random.seed(seed)
    np.random.seed(seed)
