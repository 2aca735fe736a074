"""Factory with the reference's signature (models/model_creation.py:30-191)."""
from .config import JsonConfig, adapt_legacy, is_legacy_schema
from .diffusion import GaussianSpacedDiffusion, get_named_beta_schedule, space_timesteps
from .model import Speech2GestureModel


def create_diffusion(diffusion_params, is_training):
    """model_creation.py:30-48: respacing applies only at inference."""
    if diffusion_params["type"] != "gaussian":
        raise ValueError
    betas = get_named_beta_schedule(diffusion_params["noise_schedule"], diffusion_params["diffusion_steps"])
    if not diffusion_params.get("timestep_respacing") or is_training:
        respacing = [diffusion_params["diffusion_steps"]]
    else:
        respacing = diffusion_params["timestep_respacing"]
    return GaussianSpacedDiffusion(use_timesteps=space_timesteps(diffusion_params["diffusion_steps"], respacing),
                                   betas=betas, model_var_type=diffusion_params["model_var_type"])


def create_model(d_pose, model_params, lr=1e-2, weight_decay=None, scheduler_params=None, is_training=False,
                 dtype="bf16", device="cuda", train_encoder=True):
    """model_creation.py:51-191 -> (model, diffusion, optimizer, schedule_sampler, lr_scheduler).

    Inference (is_training False): the HIP sampler model; optimizer, schedule_sampler and
    lr_scheduler are None.  Training: a training.TrainableModel (reference init, seed 0; the HA2G
    encoder trained in train mode unless train_encoder=False) with AdamW, the uniform schedule
    sampler and the configured lr schedule (the one-way or two-way decoder under
    s2g_v2, default or inpaint).  Legacy {"type","args"} model params
    (tedexp) are adapted to the flat schema first.
    """
    if is_training:
        from . import training
        from .weights import arch_from_config, init_state_dict
        if not isinstance(model_params, JsonConfig):
            model_params = JsonConfig(dict(model_params))
        if is_legacy_schema(model_params):
            model_params = adapt_legacy({"Model": model_params.to_dict()}).Model
        arch = arch_from_config(model_params, d_pose)
        seed_len = None
        if arch["type"] == "inpaint":   # model_creation.py:134-142
            seed_len = int(model_params["Generate"]["pose_seed_len"])
        model = training.TrainableModel(arch, init_state_dict(arch, seed=0), device=device, train_encoder=train_encoder,
                                        pose_seed_len=seed_len)
        diffusion = create_diffusion(model_params["Diffusion"], True)
        optimizer = training.AdamW(model, lr=lr, weight_decay=weight_decay)
        sp = scheduler_params.to_dict() if isinstance(scheduler_params, JsonConfig) else scheduler_params
        return model, diffusion, optimizer, training.UniformSampler(diffusion), training.LRScheduler(optimizer, sp)
    if not isinstance(model_params, JsonConfig):
        model_params = JsonConfig(dict(model_params))
    if is_legacy_schema(model_params):
        model_params = adapt_legacy({"Model": model_params.to_dict()}).Model
    if model_params["Encoder"]["type"] != "ha2g":
        raise ValueError
    dec = model_params["Decoder"]["type"]
    if dec not in ("oneway_cross_attention", "cross_attention"):
        raise ValueError(f"Unsupported decoder type {dec}.")
    if model_params["type"] not in ("s2g_v2", "default", "inpaint"):
        raise ValueError(f"Unsupported model_type {model_params['type']}")
    model = Speech2GestureModel(d_pose, model_params, dtype=dtype, device=device)
    diffusion = create_diffusion(model_params["Diffusion"], is_training)
    return model, diffusion, None, None, None
