"""The reference's hyperparameter surface, kept drop-in.

Two files feed ``train_aurora_gan`` in the reference:
  * ``configs/hyperparameter_config.json`` -- the HPO job description consumed by
    scripts/hyperparameter_tuning.py:97-100, :191-209 (``hyperparameter_ranges``, ``integer_parameter_ranges``,
    ``static_hyperparameters`` with string values, ``objective_metric``);
  * ``/opt/ml/input/config/hyperparameters.json`` -- the flat string->string map SageMaker hands a training
    job, coerced by moegan/sagemaker_train.py:85-102 and mapped to ``train_aurora_gan`` keyword arguments at
    sagemaker_train.py:271-294.
This module validates the first, reproduces the coercion and the keyword mapping of the second, and accepts the
``clip_weight_64`` / ``clip_weight_32`` names the HPO config actually uses (never read by sagemaker_train.py,
SURVEY.md §5) as the 16x16 / 8x8 CLIP weights.
"""
import json

# sagemaker_train.py:94-99
INT_KEYS = ("batch_size", "epochs", "kl_annealing_epochs", "lr_warmup_epochs")
FLOAT_KEYS = ("learning_rate", "beta1", "beta2", "r1_gamma", "clip_weight_16", "clip_weight_8", "kl_weight",
              "balance_weight")
# keys of the HPO config that name CLIP weights the training entry point knows under other names
CLIP_ALIASES = {"clip_weight_64": "clip_weight_16", "clip_weight_32": "clip_weight_8"}

# sagemaker_train.py:271-294: hyperparameter -> (train_aurora_gan keyword, default)
TRAIN_KWARGS = {
    "epochs": ("num_epochs", 50),
    "learning_rate": ("lr", 0.0002),
    "beta1": ("beta1", 0.5),
    "beta2": ("beta2", 0.999),
    "r1_gamma": ("r1_gamma", 10.0),
    "clip_weight_16": ("clip_weight_16", 0.1),
    "clip_weight_8": ("clip_weight_8", 0.05),
    "kl_weight": ("kl_weight", 0.001),
    "kl_annealing_epochs": ("kl_annealing_epochs", 5),
    "lr_warmup_epochs": ("lr_warmup_epochs", 3),
    "balance_weight": ("balance_weight", 0.01),
}
# fixed by the SageMaker entry point (sagemaker_train.py:287-292)
TRAIN_FIXED = {"log_interval": 100, "save_interval": 500, "gradient_accumulation_steps": 8,
               "checkpoint_activation": True, "batch_memory_limit": 20.0, "max_resolution": 16}

SCALING_TYPES = ("Auto", "Linear", "Logarithmic", "ReverseLogarithmic")


def coerce_hyperparameters(raw):
    """sagemaker_train.parse_sagemaker_parameters (:85-102): int / float keys converted, the rest passed as is.
    The HPO config's clip_weight_64 / clip_weight_32 are coerced as floats too (they are CLIP weights)."""
    params = {}
    for key, value in raw.items():
        if key in INT_KEYS:
            params[key] = int(value)
        elif key in FLOAT_KEYS or key in CLIP_ALIASES:
            params[key] = float(value)
        else:
            params[key] = value
    return params


def load_sagemaker_hyperparameters(path):
    with open(path) as f:
        return coerce_hyperparameters(json.load(f))


def train_kwargs(params, fixed=True):
    """``train_aurora_gan`` keyword arguments for coerced hyperparameters, with the SageMaker entry point's
    defaults (:271-294).  ``clip_weight_64/32`` fill ``clip_weight_16/8`` when those are absent."""
    p = dict(params)
    for alias, key in CLIP_ALIASES.items():
        if alias in p and key not in p:
            p[key] = p[alias]
    kw = {name: p.get(key, default) for key, (name, default) in TRAIN_KWARGS.items()}
    if fixed:
        kw.update(TRAIN_FIXED)
    return kw


def given_train_kwargs(params):
    """Only the ``train_aurora_gan`` keyword arguments that ``params`` actually sets (to override CLI flags)."""
    p = dict(params)
    for alias, key in CLIP_ALIASES.items():
        if alias in p and key not in p:
            p[key] = p[alias]
    return {name: p[key] for key, (name, _) in TRAIN_KWARGS.items() if key in p}


def unapplied_keys(params):
    """Keys of coerced hyperparameters that neither size the DataLoaders (batch_size) nor map to a
    ``train_aurora_gan`` keyword: reported by train_model.py instead of being dropped silently."""
    used = set(TRAIN_KWARGS) | set(CLIP_ALIASES) | {"batch_size"}
    return {k for k in params if k not in used}


def _num(x, what):
    if not isinstance(x, (int, float)) or isinstance(x, bool):
        raise ValueError(f"{what}: expected a number, got {x!r}")
    return x


def validate_hpo_config(cfg):
    """Check a configs/hyperparameter_config.json document against the schema hyperparameter_tuning.py reads;
    returns it unchanged, raises ValueError naming the first problem."""
    if not isinstance(cfg, dict):
        raise ValueError("config must be a JSON object")
    for sect, integer in (("hyperparameter_ranges", False), ("integer_parameter_ranges", True)):
        for name, r in cfg.get(sect, {}).items():
            if not isinstance(r, dict):
                raise ValueError(f"{sect}.{name}: expected an object")
            lo, hi = _num(r.get("min_value"), f"{sect}.{name}.min_value"), _num(r.get("max_value"),
                                                                                 f"{sect}.{name}.max_value")
            if integer and (int(lo) != lo or int(hi) != hi):
                raise ValueError(f"{sect}.{name}: integer range with non-integer bounds")
            if lo > hi:
                raise ValueError(f"{sect}.{name}: min_value > max_value")
            st = r.get("scaling_type", "Auto")
            if st not in SCALING_TYPES:
                raise ValueError(f"{sect}.{name}.scaling_type: {st!r} not in {SCALING_TYPES}")
            if st in ("Logarithmic", "ReverseLogarithmic") and lo <= 0:
                raise ValueError(f"{sect}.{name}: logarithmic scaling needs min_value > 0")
    static = cfg.get("static_hyperparameters", {})
    for k, v in static.items():
        if not isinstance(v, str):
            raise ValueError(f"static_hyperparameters.{k}: SageMaker passes strings, got {type(v).__name__}")
    obj = cfg.get("objective_metric")
    if obj is not None:
        if not isinstance(obj, dict) or "name" not in obj or obj.get("type") not in ("Minimize", "Maximize"):
            raise ValueError("objective_metric: needs a name and type Minimize|Maximize")
    return cfg


def load_hpo_config(path):
    with open(path) as f:
        return validate_hpo_config(json.load(f))


def static_train_kwargs(cfg):
    """The keyword arguments one HPO training job starts from: the static hyperparameters, coerced as the
    training container would (ranges are filled in per job by the tuner)."""
    return train_kwargs(coerce_hyperparameters(cfg.get("static_hyperparameters", {})))
