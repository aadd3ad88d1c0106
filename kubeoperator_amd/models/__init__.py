"""Model families of the bundled training chart: Llama-3 (RMSNorm/RoPE/GQA/SwiGLU) and GPT-2."""
from .config import CONFIGS, ModelConfig, get_config
from .gpt2 import GPT2
from .llama import Llama


def build_model(cfg: ModelConfig, tp=None):
    """``tp``: a ``parallel.tensor.TPContext`` (tensor parallelism is implemented for the Llama family)."""
    if cfg.arch == "llama":
        return Llama(cfg, tp)
    if cfg.arch == "gpt2":
        if tp is not None and tp.size > 1:
            raise ValueError("tensor parallelism is implemented for the Llama family")
        return GPT2(cfg)
    raise ValueError(f"unknown architecture {cfg.arch}")


__all__ = ["CONFIGS", "ModelConfig", "get_config", "Llama", "GPT2", "build_model"]
