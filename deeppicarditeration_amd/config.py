"""YAML configuration surface of the reference (`picard/config.py`), without yacs (not in this
image): the same default schema, `BASE:` chaining with `NAME` joining (config.py:229-257) and
`KEY VALUE` command-line overrides (config.py:259-262), so the reference's experiment YAMLs load
unchanged.  Keys added by this build (all under DATA): BACKEND ("hip"), SEED, EULER_STEPS,
POINTS_PER_CALL.
"""
import ast
import copy
import os
from typing import List

import yaml


class CfgNode(dict):
    """Attribute-access dict with yacs-like merge / freeze / dump."""

    def __init__(self, init=None, new_allowed=False):
        super().__init__()
        object.__setattr__(self, "_frozen", False)
        object.__setattr__(self, "_new_allowed", new_allowed)
        for k, v in (init or {}).items():
            self[k] = CfgNode(v, new_allowed=True) if isinstance(v, dict) and not isinstance(v, CfgNode) else v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        if self._frozen:
            raise AttributeError(f"config is frozen: cannot set {k}")
        self[k] = v

    def freeze(self):
        object.__setattr__(self, "_frozen", True)
        for v in self.values():
            if isinstance(v, CfgNode):
                v.freeze()

    def clone(self):
        return copy.deepcopy(self)

    def to_dict(self):
        return {k: v.to_dict() if isinstance(v, CfgNode) else v for k, v in self.items()}

    def dump(self):
        return yaml.safe_dump(self.to_dict(), sort_keys=False)

    def merge_from_other_cfg(self, other, path=""):
        for k, v in other.items():
            full = f"{path}{k}"
            if k not in self:
                if not self._new_allowed:
                    raise KeyError(f"Non-existent config key: {full}")
                self[k] = CfgNode(v, new_allowed=True) if isinstance(v, dict) else v
                continue
            if isinstance(self[k], CfgNode) and isinstance(v, dict):
                self[k].merge_from_other_cfg(v, full + ".")
            else:
                self[k] = _coerce(v, self[k], full)

    def merge_from_list(self, opts: List[str]):
        if len(opts) % 2:
            raise ValueError(f"override list needs KEY VALUE pairs: {opts}")
        for key, raw in zip(opts[0::2], opts[1::2]):
            node = self
            parts = key.split(".")
            for p in parts[:-1]:
                if p not in node:
                    raise KeyError(f"Non-existent config key: {key}")
                node = node[p]
            if parts[-1] not in node and not node._new_allowed:
                raise KeyError(f"Non-existent config key: {key}")
            node[parts[-1]] = _coerce(_literal(raw), node.get(parts[-1]), key)


def _literal(v):
    if isinstance(v, str):
        try:
            return ast.literal_eval(v)
        except (ValueError, SyntaxError):
            return v
    return v


def _coerce(v, old, key):
    v = _literal(v)
    if v == "None":
        v = None
    if isinstance(v, dict):
        return CfgNode(v, new_allowed=True)
    if old is None or v is None:
        return v
    if isinstance(old, bool) or isinstance(v, bool):
        return v
    if isinstance(old, (int, float)) and isinstance(v, (int, float)):
        return type(old)(v) if isinstance(old, float) else v
    if isinstance(old, (list, tuple)) and isinstance(v, (list, tuple)):
        return list(v)
    return v


def _N(d=None, new_allowed=False):
    return CfgNode(d or {}, new_allowed=new_allowed)


def get_default_cfg() -> CfgNode:
    """The reference's `_C` (picard/config.py:9-116) + this build's DATA keys."""
    C = _N()
    C.BASE = None
    C.FORCE = False
    C.NAME = "exp"
    C.EQUATION = _N({"cls": "AllenCahnEquation"})
    C.EQUATION.kwargs = _N(new_allowed=True)
    C.METHOD = _N({"cls": "Picard", "num_v_samples": 16, "K": 20, "dt": 0.005, "num_sub_iter": 100})
    C.PICARD = _N({"N": 1, "FORMULA": None})
    C.TRAIN = _N({"BATCH_SIZE": 2048, "N_EPOCHS": 1, "SUPERVISE_GRADIENT": None, "SUPERVISE_HESSIAN": None,
                  "NUM_HESS_SAMPLES": -1})
    C.TRAIN.LOSS = _N({"beta": 0.0, "use_aux_loss": False, "weight_aux_loss": 0.1})
    C.TRAIN.LOSS.SCALER = _N({"cls": None})
    C.TRAIN.LOSS.SCALER.kwargs = _N(new_allowed=True)
    C.TRAIN.LOSS.FN = _N({"cls": None})
    C.TRAIN.LOSS.FN.kwargs = _N(new_allowed=True)
    C.TRAIN.OPTIMIZER = _N({"cls": "Adam"})
    C.TRAIN.OPTIMIZER.kwargs = _N(new_allowed=True)
    C.TRAIN.OPTIMIZER.SCHEDULER = _N({"cls": None})
    C.TRAIN.OPTIMIZER.SCHEDULER.kwargs = _N(new_allowed=True)
    C.TRAIN.OPTIMIZER.SCHEDULER.config = _N(new_allowed=True)
    C.NETWORK = _N({"cls": None, "TYPE": "Value", "NEURONS": [10, 10], "ACTIVATIONS": ["Tanh", "Tanh"], "BOUND": None,
                    "RELOAD": False, "USE_T_EMBEDDING": False, "PISGRADNET": False, "PRETRAIN_PATH": None})
    C.NETWORK.kwargs = _N(new_allowed=True)
    C.DATA = _N({"SAVE": False, "ONLINE": True, "TRAIN_FILE": "", "N_WORKERS": 1, "DATA_SIZE": 2048 * 5000,
                 "NEW_SAMPLING": False, "N_BUFFER": None, "RESERVED_MEMORY": None, "PREFETCH_FACTOR": None,
                 "DEVICE": None, "FLOAT": "float", "EXACT": False, "SHUFFLE": None, "PRELOAD": False,
                 "PRELOAD_N_WORKERS": None, "SAMPLE_BOUND": None, "ESTIMATE_TERMINAL": "OU_ByGx",
                 "ESTIMATE_INTEGRAL": "OU_Simple", "ESTIMATE_DELTA_T": 0.0,
                 # this build
                 "BACKEND": "hip", "SEED": 0, "EULER_STEPS": 50, "POINTS_PER_CALL": 512})
    C.DATA.kwargs = _N(new_allowed=True)
    C.DATA.MEMORY = _N({"RESERVED": None, "REDUCE_FACTOR": 1.0, "REUSE": 9999999})
    C.DATA.HESSIAN_APPROXIMATION = _N({"method": None})
    C.DATA.HESSIAN_APPROXIMATION.kwargs = _N(new_allowed=True)
    C.LOGGING = _N({"LOGGER": "wandb", "TENSORBOARD_DIR": "tensorboard"})
    C.LOGGING.kwargs = _N({"project": "picard", "offline": False}, new_allowed=True)
    C.EVAL = _N({"L2_N_POINTS": 10_000, "FREQ": None, "BATCH_SIZE": None, "TEST_GRAD": False, "TEST_HESSIAN": False})
    return C


def _read_file_only(path):
    with open(path) as f:
        return CfgNode(yaml.safe_load(f) or {}, new_allowed=True)


def load_cfg(cfg_file: str, override: List[str] = None) -> CfgNode:
    """picard/config.py:242-266: BASE chain (deepest first), NAME joined with '_', overrides."""
    top = _read_file_only(cfg_file)
    bases = []
    node, here = top, os.path.dirname(os.path.abspath(cfg_file))
    while node.get("BASE") is not None:
        path = node.BASE
        if not os.path.exists(path):  # the reference resolves BASE from the CWD; also accept file-relative
            path = os.path.join(here, node.BASE)
        here = os.path.dirname(os.path.abspath(path))
        node = _read_file_only(path)
        bases.append(node)
    cfg = get_default_cfg()
    names = []
    for b in reversed(bases):
        cfg.merge_from_other_cfg(b)
        if "NAME" in b:
            names.append(b.NAME)
    cfg.merge_from_other_cfg(top)
    cfg.NAME = "_".join(names + [top.get("NAME", cfg.NAME)])
    cfg.pop("BASE", None)
    if override:
        for item in override:
            if item.startswith("BASE") or item.startswith("--BASE"):
                raise ValueError("override should not contain BASE")
        cfg.merge_from_list(override)
    if cfg.DATA.RESERVED_MEMORY is not None:  # config.py:119-125
        if cfg.DATA.MEMORY.RESERVED is None:
            cfg.DATA.MEMORY.RESERVED = cfg.DATA.RESERVED_MEMORY
        else:
            raise ValueError("Both RESERVED_MEMORY and MEMORY.RESERVED are set.")
    cfg.freeze()
    return cfg
