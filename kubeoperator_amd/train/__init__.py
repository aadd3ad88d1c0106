"""Training loop of the bundled PyTorch-ROCm chart (trainer, data sources, checkpointing)."""
from .data import SyntheticTokens, TokenFileDataset
from .trainer import TrainConfig, Trainer, lr_at

__all__ = ["SyntheticTokens", "TokenFileDataset", "TrainConfig", "Trainer", "lr_at"]
