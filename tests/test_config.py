"""YAML config surface (picard/config.py) and the `picard train` front end — CPU only."""
import glob
import os

import pytest

from deeppicarditeration_amd.config import get_default_cfg, load_cfg
from deeppicarditeration_amd.main import main

REF_SCRIPTS = "/root/reference/scripts"


def _write(p, text):
    p.write_text(text)
    return str(p)


def test_defaults_match_reference_schema():
    c = get_default_cfg()
    assert c.PICARD.N == 1 and c.TRAIN.BATCH_SIZE == 2048 and c.DATA.DATA_SIZE == 2048 * 5000
    assert c.DATA.ESTIMATE_TERMINAL == "OU_ByGx" and c.DATA.ESTIMATE_INTEGRAL == "OU_Simple"
    assert c.NETWORK.TYPE == "Value" and c.DATA.BACKEND == "hip"


def test_base_chain_name_join_and_overrides(tmp_path):
    _write(tmp_path / "base.yaml", "NAME: base\nEQUATION:\n  cls: Cha\n  kwargs: {nx: 10, alpha: 1.0, k: 5.0}\n"
                                   "PICARD: {N: 8}\nDATA: {PREFETCH_FACTOR: None, kwargs: {n_estimate_terminal: 64}}\n")
    top = _write(tmp_path / "top.yaml", "BASE: base.yaml\nNAME: top\nTRAIN: {N_EPOCHS: 3}\n")
    cwd = os.getcwd()
    try:
        os.chdir(tmp_path)
        cfg = load_cfg(top, ["PICARD.N", "2", "TRAIN.LOSS.beta", "1", "EQUATION.kwargs.T", "0.5"])
    finally:
        os.chdir(cwd)
    assert cfg.NAME == "base_top"
    assert cfg.PICARD.N == 2 and cfg.TRAIN.N_EPOCHS == 3
    assert cfg.TRAIN.LOSS.beta == 1.0 and isinstance(cfg.TRAIN.LOSS.beta, float)
    assert cfg.EQUATION.kwargs == {"nx": 10, "alpha": 1.0, "k": 5.0, "T": 0.5}
    assert cfg.DATA.PREFETCH_FACTOR is None and cfg.DATA.kwargs.n_estimate_terminal == 64
    assert "BASE" not in cfg
    with pytest.raises(AttributeError):
        cfg.NAME = "x"


def test_unknown_key_and_base_override_rejected(tmp_path):
    bad = _write(tmp_path / "bad.yaml", "NAME: x\nTRAIN: {NOT_A_KEY: 1}\n")
    with pytest.raises(KeyError):
        load_cfg(bad)
    ok = _write(tmp_path / "ok.yaml", "NAME: x\n")
    with pytest.raises(KeyError):
        load_cfg(ok, ["PICARD.NOPE", "1"])
    with pytest.raises(ValueError):
        load_cfg(ok, ["BASE", "a.yaml"])


def test_reserved_memory_compat(tmp_path):
    f = _write(tmp_path / "m.yaml", "NAME: x\nDATA: {RESERVED_MEMORY: 3.0}\n")
    assert load_cfg(f).DATA.MEMORY.RESERVED == 3.0
    g = _write(tmp_path / "g.yaml", "NAME: x\nDATA: {RESERVED_MEMORY: 3.0, MEMORY: {RESERVED: 1.0}}\n")
    with pytest.raises(ValueError):
        load_cfg(g)


@pytest.mark.skipif(not os.path.isdir(REF_SCRIPTS), reason="reference experiment YAMLs not present")
@pytest.mark.parametrize("path", sorted(glob.glob(f"{REF_SCRIPTS}/**/*.yaml", recursive=True)))
def test_reference_yamls_load(path):
    """Every experiment YAML the reference ships loads into this schema unchanged (read as data)."""
    cwd = os.getcwd()
    try:
        os.chdir(os.path.dirname(path))
        cfg = load_cfg(os.path.basename(path), ["PICARD.N", "1"])
    finally:
        os.chdir(cwd)
    assert cfg.PICARD.N == 1 and cfg.NAME


def test_cli_usage_and_missing_file(capsys):
    assert main([]) == 2
    with pytest.raises(SystemExit):
        main(["train", "/nonexistent/cfg.yaml"])


def test_runner_rejects_out_of_scope_methods(tmp_path):
    from deeppicarditeration_amd.runner import PicardRunner
    f = _write(tmp_path / "d.yaml", f"NAME: {tmp_path}/d\nEQUATION:\n  cls: Cha\n  kwargs: {{nx: 4, alpha: 1.0}}\n"
                                    "METHOD: {cls: Diffusion}\n")
    with pytest.raises(NotImplementedError):
        PicardRunner(load_cfg(f), device="cpu")



def test_picard_console_entry_point(capsys):
    """pyproject.toml exposes `picard` -> deeppicarditeration_amd.main:main (reference pyproject.toml:25-26)."""
    import importlib
    import tomli
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "pyproject.toml"), "rb") as f:
        target = tomli.load(f)["project"]["scripts"]["picard"]
    mod, fn = target.split(":")
    main = getattr(importlib.import_module(mod), fn)
    assert main([]) == 2 and "picard train" in capsys.readouterr().out
    with pytest.raises(SystemExit):
        main(["train", "/nonexistent.yaml"])
