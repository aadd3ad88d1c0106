"""Model families of the bundled training chart: Llama-3 (RMSNorm/RoPE/GQA/SwiGLU) and GPT-2."""
from .config import CONFIGS, ModelConfig, get_config
from .gpt2 import GPT2
from .llama import Llama


def build_model(cfg: ModelConfig):
    if cfg.arch == "llama":
        return Llama(cfg)
    if cfg.arch == "gpt2":
        return GPT2(cfg)
    raise ValueError(f"unknown architecture {cfg.arch}")


__all__ = ["CONFIGS", "ModelConfig", "get_config", "Llama", "GPT2", "build_model"]
