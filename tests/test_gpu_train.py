"""End-to-end `picard train` on the GPU: tiny Picard runs whose labels come from the HIP path and
stay on the device."""
import json

import pytest
import torch

from deeppicarditeration_amd.config import load_cfg
from deeppicarditeration_amd.runner import PicardRunner

pytestmark = pytest.mark.gpu

CHA = """NAME: {name}
EQUATION:
  cls: Cha
  kwargs: {{nx: 8, alpha: 1.0, k: 5.0, T: 1.0}}
PICARD: {{N: 3}}
FORCE: true
DATA:
  DATA_SIZE: 1024
  POINTS_PER_CALL: 384
  EULER_STEPS: 4
  kwargs: {{t_always_uniform: true, n_estimate_terminal: 1024, n_estimate_integral: 1024}}
TRAIN:
  N_EPOCHS: 16
  BATCH_SIZE: 128
  SUPERVISE_GRADIENT: true
  LOSS: {{beta: 0.0, SCALER: {{cls: FixedLossScaler, kwargs: {{fixed_weight: 0.1}}}}}}
  OPTIMIZER: {{kwargs: {{lr: 0.003}}}}
NETWORK:
  NEURONS: [32, 32]
  ACTIVATIONS: [ELU, ELU]
  BOUND: None
  RELOAD: true
EVAL: {{L2_N_POINTS: 512}}
"""


def test_picard_train_cha_device_labels(tmp_path):
    f = tmp_path / "cha.yaml"
    f.write_text(CHA.format(name=tmp_path / "run"))
    runner = PicardRunner(load_cfg(str(f)))
    hist = runner.run()
    assert [h["iter"] for h in hist] == [1, 2, 3]
    assert all(h["labels"] == 1024 for h in hist)
    for i in (1, 2, 3):
        sd = torch.load(tmp_path / "run" / f"model_{i}.pt", weights_only=True)
        assert all(torch.isfinite(v).all() for v in sd.values())
    rel = [h["rel_l2_u"] for h in hist]
    assert all(r is not None and r == r for r in rel)
    # the Picard iterates approach the exact Burgers solution sigmoid(t + k' sum x)
    print("rel_l2_u per iteration", rel)
    assert max(rel) < 0.6 and min(rel) < 0.3, rel
    lines = (tmp_path / "run" / "history.jsonl").read_text().splitlines()
    assert [json.loads(l)["iter"] for l in lines] == [1, 2, 3]


def test_label_buffer_is_device_resident(tmp_path):
    f = tmp_path / "cha.yaml"
    f.write_text(CHA.format(name=tmp_path / "run2"))
    runner = PicardRunner(load_cfg(str(f), ["PICARD.N", "1"]))
    runner.i = 1
    tx, y = runner.labels()
    assert tx.is_cuda and y.is_cuda and tx.shape == (1024, 9) and y.shape == (1024, 9)
    assert torch.isfinite(y).all()


GBM_HESS = """NAME: {name}
EQUATION:
  cls: GBMEquationComplexExact
  kwargs: {{nx: 100, alpha: 1.0, T: 1.0}}
PICARD: {{N: 2}}
FORCE: true
DATA:
  DATA_SIZE: 256
  POINTS_PER_CALL: 128
  EULER_STEPS: 4
  kwargs: {{t_always_uniform: true, n_estimate_terminal: 128, n_estimate_integral: 128}}
TRAIN:
  N_EPOCHS: 2
  BATCH_SIZE: 64
  SUPERVISE_GRADIENT: true
  SUPERVISE_HESSIAN: true
  NUM_HESS_SAMPLES: 500
  LOSS: {{beta: 0.0, SCALER: {{cls: FixedHessianLossScaler, kwargs: {{fixed_gradient_weight: 0.1, fixed_hessian_weight: 0.01}}}}}}
NETWORK:
  NEURONS: [32, 32]
  ACTIVATIONS: [ELU, ELU]
  BOUND: None
  RELOAD: true
EVAL: {{L2_N_POINTS: 256}}
"""


def test_picard_train_gbm_hessian_supervision(tmp_path):
    """TRAIN.SUPERVISE_HESSIAN: Malliavin Hessian labels (n, 1 + nx + nx^2) from the device path
    feed the gradient + Hessian loss of PicardSolutionGradientHessianWrapper."""
    f = tmp_path / "gbm.yaml"
    f.write_text(GBM_HESS.format(name=tmp_path / "run"))
    runner = PicardRunner(load_cfg(str(f)))
    runner.i = 1
    tx, y = runner.labels()
    assert y.shape == (256, 1 + 100 + 100 * 100) and torch.isfinite(y).all()
    h = y[:, 101:].reshape(-1, 100, 100)
    assert torch.equal(h, h.transpose(1, 2))
    runner.i = 0
    hist = runner.run()
    assert [h_["iter"] for h_ in hist] == [1, 2]
    assert all(h_["loss"] == h_["loss"] for h_ in hist) and all(h_["rel_l2_u"] is not None for h_ in hist)


def test_picard_train_saves_reference_label_files(tmp_path):
    """DATA.SAVE: true writes each iteration's labels as the reference's data_iter_{i}/split_00.h5
    (datasets tx and u_ux, DATA.FLOAT), equal to the device labels of that iteration."""
    import numpy as np
    from deeppicarditeration_amd import h5
    from deeppicarditeration_amd.h5 import H5Dataset, read_dataset
    try:
        h5._load()
    except RuntimeError as e:
        pytest.skip(str(e))
    f = tmp_path / "cha.yaml"
    f.write_text(CHA.format(name=tmp_path / "run_save").replace("  DATA_SIZE: 1024", "  DATA_SIZE: 1024\n  SAVE: true")
                 .replace("PICARD: {N: 3}", "PICARD: {N: 2}"))
    runner = PicardRunner(load_cfg(str(f)))
    seen = {}
    orig = runner.labels

    def labels():
        tx, y = orig()
        seen[runner.i] = (tx.cpu().numpy(), y.cpu().numpy())
        return tx, y

    runner.labels = labels
    runner.run()
    for i in (1, 2):
        p = tmp_path / "run_save" / f"data_iter_{i}" / "split_00.h5"
        tx, y = read_dataset(p, "tx"), read_dataset(p, "u_ux")
        assert tx.dtype == np.float32 and tx.shape == (1024, 9) and y.shape == (1024, 9)
        assert np.array_equal(tx, seen[i][0]) and np.array_equal(y, seen[i][1])
        batches = list(H5Dataset(p, 256, ["tx", "u_ux"]))
        assert len(batches) == 4 and torch.equal(batches[1][1], torch.from_numpy(seen[i][1][256:512]))
