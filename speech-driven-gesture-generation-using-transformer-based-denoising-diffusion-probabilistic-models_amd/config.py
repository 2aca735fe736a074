"""Config-JSON surface of the reference: JsonConfig + the legacy (tedexp) schema adapter.

JsonConfig mirrors utils/json_config.py:6-125: a ``dict`` with attribute access,
nested dicts become JsonConfig, ``Meta.name`` defaults to the file stem, and
``dump``/``to_dict`` round-trip to JSON.  Missing keys raise ``KeyError`` from
``__getattr__`` like the reference (json_config.py:63-64).
"""
import copy
import json
import os


class JsonConfig(dict):
    Indent = 4

    def __init__(self, *args, **kwargs):
        super().__init__()
        assert len(args) == 0 or len(kwargs) == 0, \
            "[JsonConfig]: Cannot initialize with position parameters and named parameters at the same time."
        if args:
            assert len(args) == 1, "[JsonConfig]: Need one positional parameters, found two."
            src = args[0]
        else:
            src = kwargs
        if isinstance(src, str):
            stem = os.path.splitext(os.path.basename(src))[0]
            with open(src) as f:
                src = json.load(f)
            meta = src.setdefault("Meta", {})
            meta.setdefault("name", stem)
        if not isinstance(src, dict):
            raise TypeError(f"[JsonConfig]: Do not support given input with type {type(src)}")
        for k, v in src.items():
            super().__setitem__(k, JsonConfig(v) if isinstance(v, dict) else v)

    def __getattr__(self, attr):
        return super().__getitem__(attr)

    def __getstate__(self):
        return self.__dict__

    def __setstate__(self, d):
        self.__dict__ = d

    def to_dict(self):
        return {k: (v.to_dict() if isinstance(v, JsonConfig) else v)
                for k, v in self.items() if not k.startswith("__")}

    def dump(self, path):
        with open(path, "w") as f:
            json.dump(self.to_dict(), f, indent=JsonConfig.Indent)

    def __str__(self):
        return json.dumps(self.to_dict(), indent=JsonConfig.Indent)


def is_legacy_schema(model_params):
    """tedexp-style configs nest every block as {"type", "args"} (configs/tedexp-ours.json:17-67)."""
    return "Model" in model_params and isinstance(model_params["Model"], dict) \
        and "args" in model_params["Model"]


def adapt_legacy(config):
    """Return a flat-schema copy of a tedexp-style config.

    configs/tedexp-ours.json keeps d_model/dropout under Model.Model.args and the
    decoder/diffusion options under *.args; create_model reads them flat
    (models/model_creation.py:63-131, KeyError('d_model') on the legacy file).
    The adapter lifts every ``args`` dict into its block and promotes
    Model.Model.{type, args} to Model.{type, d_model, dropout_prob}.
    """
    cfg = copy.deepcopy(config.to_dict() if isinstance(config, JsonConfig) else dict(config))
    model = cfg.get("Model", {})
    if not is_legacy_schema(model):
        return JsonConfig(cfg)
    flat = {}
    inner = model["Model"]
    flat["type"] = inner["type"]
    flat.update(inner.get("args", {}))
    for block in ("Encoder", "Decoder", "Diffusion"):
        if block in model:
            b = {"type": model[block]["type"]}
            b.update(model[block].get("args", {}))
            flat[block] = b
    gen = dict(cfg.get("Generate", {}))
    if "pose_seed_len" in flat:
        gen.setdefault("pose_seed_len", flat["pose_seed_len"])
    flat["Generate"] = gen
    cfg["Model"] = flat
    data = cfg.get("Data", {})
    if "args" in data:
        d = {"type": data.get("type")}
        d.update(data["args"])
        cfg["Data"] = d
    return JsonConfig(cfg)


def load_config(path):
    """Load a reference config (either schema) into the flat schema create_model reads."""
    return adapt_legacy(JsonConfig(path))
