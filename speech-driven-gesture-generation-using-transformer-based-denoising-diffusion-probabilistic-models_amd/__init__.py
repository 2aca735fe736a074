"""MI355X-native gesture-diffusion sampler.

Drop-in for the inference hot path of "Speech-driven Gesture Generation using
Transformer-based Denoising Diffusion Probabilistic Models": the DDPM/DDIM reverse
loop (models/modules/gaussian_diffusion.py, respace.py) around the transformer
denoiser (models/model.py, models/nn.py, models/modules/transformer.py), behind
the reference's create_model / Generator / JsonConfig surface.

The decoder and the diffusion update run as hand-written gfx950 kernels in
libggd.so (csrc/), reached through its C ABI (include/ggd.h) with ctypes.
"""
from .config import JsonConfig, adapt_legacy, load_config
from .diffusion import (GaussianDiffusion, GaussianSpacedDiffusion, InpaintDenoise, get_named_beta_schedule,
                        space_timesteps)
from .generator import Generator
from .model import Speech2GestureModel, sync_all
from .model_creation import create_diffusion, create_model
from .weights import arch_from_config, count_parameters, init_state_dict, parameter_shapes

__all__ = [
    "JsonConfig", "adapt_legacy", "load_config", "GaussianDiffusion", "GaussianSpacedDiffusion",
    "InpaintDenoise", "get_named_beta_schedule", "space_timesteps", "Generator", "Speech2GestureModel",
    "create_diffusion", "create_model", "sync_all", "arch_from_config", "count_parameters", "init_state_dict",
    "parameter_shapes",
]
