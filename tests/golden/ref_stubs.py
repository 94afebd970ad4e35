"""Stand-ins for the third-party modules the reference imports but this image lacks (yacs,
lightning, h5py, tensorboardX), and a synthetic `picard` package whose __path__ points at a
reference source tree, bypassing picard/__init__.py (which pulls wandb) — SURVEY.md §8c.  Used
only in the build container, by the fixture generators and by the reference-binding check; never
on the GPU box."""
import sys
import types

import torch


def install_stubs(picard_dir):
    class CfgNode(dict):
        def __init__(self, init=None, new_allowed=False, **kw):
            super().__init__(init or {})

        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

        def __setattr__(self, k, v):
            self[k] = v

    yacs = types.ModuleType("yacs")
    yacs_cfg = types.ModuleType("yacs.config")
    yacs_cfg.CfgNode = CfgNode
    yacs.config = yacs_cfg
    sys.modules["yacs"] = yacs
    sys.modules["yacs.config"] = yacs_cfg

    class LightningModule(torch.nn.Module):
        def save_hyperparameters(self, *a, **k):
            pass

        def log(self, *a, **k):
            pass

        def log_dict(self, *a, **k):
            pass

    class _Dummy:
        def __init__(self, *a, **k):
            pass

    pl = types.ModuleType("lightning")
    plp = types.ModuleType("lightning.pytorch")
    for mod in (pl, plp):
        mod.LightningModule = LightningModule
        mod.LightningDataModule = _Dummy
        mod.Callback = _Dummy
        mod.Trainer = _Dummy
    pl.pytorch = plp
    fab = types.ModuleType("lightning.fabric")
    fabu = types.ModuleType("lightning.fabric.utilities")
    fabw = types.ModuleType("lightning.fabric.utilities.warnings")
    fabw.PossibleUserWarning = UserWarning
    plu = types.ModuleType("lightning.pytorch.utilities")
    plut = types.ModuleType("lightning.pytorch.utilities.types")
    plut.EVAL_DATALOADERS = object
    for name, mod in {
        "lightning": pl, "lightning.pytorch": plp, "lightning.fabric": fab,
        "lightning.fabric.utilities": fabu, "lightning.fabric.utilities.warnings": fabw,
        "lightning.pytorch.utilities": plu, "lightning.pytorch.utilities.types": plut,
    }.items():
        sys.modules[name] = mod
    h5 = types.ModuleType("h5py")
    h5.File = _Dummy
    sys.modules["h5py"] = h5
    tbx = types.ModuleType("tensorboardX")
    tbx.SummaryWriter = _Dummy
    sys.modules["tensorboardX"] = tbx
    pkg = types.ModuleType("picard")
    pkg.__path__ = [str(picard_dir)]
    sys.modules["picard"] = pkg
    return CfgNode
