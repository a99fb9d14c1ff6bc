"""``plot_loss_curves`` from the course helper_functions (MAIN.ipynb:3856, :3891, :4593)."""
from __future__ import annotations

from typing import Dict, List


def plot_loss_curves(results: Dict[str, List[float]], save_path: str = None):
    import matplotlib

    if save_path:
        matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    loss, test_loss = results["train_loss"], results["test_loss"]
    acc, test_acc = results["train_acc"], results["test_acc"]
    epochs = range(len(loss))
    plt.figure(figsize=(15, 7))
    plt.subplot(1, 2, 1)
    plt.plot(epochs, loss, label="train_loss")
    plt.plot(epochs, test_loss, label="test_loss")
    plt.title("Loss")
    plt.xlabel("Epochs")
    plt.legend()
    plt.subplot(1, 2, 2)
    plt.plot(epochs, acc, label="train_accuracy")
    plt.plot(epochs, test_acc, label="test_accuracy")
    plt.title("Accuracy")
    plt.xlabel("Epochs")
    plt.legend()
    if save_path:
        plt.savefig(save_path)
        plt.close()
